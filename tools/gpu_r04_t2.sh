#!/bin/bash
# r04: GPU parity of the box/phase kernels after the far-off / batched exact-pass change, the pair
# kernel's phase stamps, isolated kernel times, then the config-2 bench (no CPU / LC / B=109 / host legs).
set -o pipefail
mkdir -p gpurun_out
T=${1:-t2}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_palette.py \
  tests/test_gpu_parity.py > gpurun_out/pytest_${T}.log 2>&1 || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -2 gpurun_out/pytest_${T}.log
CSM_LIB=roborts-edu-slam_amd/lib/libroborts_csm-btrace.so timeout -k 10 200 python tools/box_trace.py \
  > gpurun_out/box_trace_${T}.json 2> gpurun_out/box_trace_${T}.err || { tail -20 gpurun_out/box_trace_${T}.err; exit 1; }
cat gpurun_out/box_trace_${T}.json
for l in 0 1; do timeout -k 10 200 python tools/box_kbench.py --level $l >> gpurun_out/kbench_${T}.txt 2>&1 || exit $?; done
CSM_LIB=roborts-edu-slam_amd/lib/libroborts_csm-ilp0.so timeout -k 10 200 python tools/box_kbench.py >> gpurun_out/kbench_${T}.txt 2>&1 || exit $?
grep '^{' gpurun_out/kbench_${T}.txt
timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs > gpurun_out/bench_${T}.json \
  2> gpurun_out/bench_${T}.err || { tail -20 gpurun_out/bench_${T}.err; exit 1; }
python3 - gpurun_out/bench_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step finish", round(d["finish_ms_per_step"], 3))
for k in d["kernels"]:
    if k["name"].startswith(("score_", "finish_kernel")):
        print(" ", k["name"], k["launches"], round(k["total_ms"] / k["launches"], 4))
PY
