#!/bin/bash
# r04: the early-completion mismatch (stress_ties) with the default library and with the
# per-block system-release variant (CSM_FAST_SYS_RELEASE), profiling off and on, then the
# variant's cost on the config-2 line.
set -o pipefail
mkdir -p gpurun_out
T=${1:-s4}
V=roborts-edu-slam_amd/lib/libroborts_csm-fence.so
for lib in "" $V; do
  for pr in 0 1; do
    CSM_LIB=$lib timeout -k 10 200 python tools/stress_ties.py --iters 60 --profiling $pr >> gpurun_out/stress_${T}.txt 2>&1 \
      || { tail -5 gpurun_out/stress_${T}.txt; exit 1; }
    echo "lib=${lib:-default} profiling=$pr $(tail -1 gpurun_out/stress_${T}.txt | cut -c1-200)"
  done
done
for lib in "" $V "" $V; do
  CSM_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs > gpurun_out/bench_${T}.json \
    2> gpurun_out/bench_${T}.err || { tail -20 gpurun_out/bench_${T}.err; exit 1; }
  python3 - gpurun_out/bench_${T}.json "${lib:-default}" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
fin = [k for k in d["kernels"] if k["name"].startswith("finish:fast")]
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step",
      [(k["name"], round(k["total_ms"] / max(1, k["launches"]) * 1e3, 1)) for k in fin])
PY
done
