#!/bin/bash
# r04: 16 strip copies (no byte alignment in the pair kernel) and the paired phase flush, as variant
# libraries: parity of the box/palette/phase tests under each, isolated kernel times, config-2 lines.
set -o pipefail
mkdir -p gpurun_out
T=${1:-s10}
L16=roborts-edu-slam_amd/lib/libroborts_csm-s16.so
LPF=roborts-edu-slam_amd/lib/libroborts_csm-pflush.so
for lib in $L16 $LPF; do
  CSM_LIB=$lib timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_palette.py \
    tests/test_gpu_parity.py -k "palette or box or headline or phase or three_level or host_signal" > gpurun_out/pytest_${T}.log 2>&1
  rc=$?; echo "$lib $(tail -1 gpurun_out/pytest_${T}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_${T}.log; exit $rc; }
done
out=gpurun_out/kbench_${T}.txt; : > $out
for lib in "" $L16 "" $L16; do echo "# lib=$lib" >> $out; CSM_LIB=$lib timeout -k 10 200 python tools/box_kbench.py >> $out 2>&1 || exit $?; done
for lib in "" $LPF; do echo "# lib=$lib level1" >> $out; CSM_LIB=$lib timeout -k 10 200 python tools/box_kbench.py --level 1 >> $out 2>&1 || exit $?; done
grep '^[{#]' $out | cut -c1-220
for lib in "" $L16 "" $L16; do
  CSM_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs > gpurun_out/ab_${T}.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}.json "${lib:-default}" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
k = {x["name"]: x for x in d["kernels"]}
g = lambda n: round(k[n]["total_ms"] / max(1, k[n]["launches"]) * 1e3, 1) if n in k else None
print(sys.argv[2][-20:], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step box", g("score_box_pair_kernel<13,all>"),
      "entry->first", g("host:entry->first_launch"), "prep", g("host:first:prepare+alloc"))
PY
done
