#!/bin/bash
# r04: reused LevelRuns + seal classification inside the parallel completion: stress, driver parity
# tests, repeated config-2 lines; then the pair box kernel's phase stamps (btrace variant).
set -o pipefail
mkdir -p gpurun_out
T=${1:-s9}
for env in "X=0" "CSM_FIRST_WINDOWS=0"; do
  env $env CSM_DEBUG_FIN=1 timeout -k 10 200 python tools/stress_ties.py --iters 40 > gpurun_out/stress_${T}.txt 2>&1 || { tail -5 gpurun_out/stress_${T}.txt; exit 1; }
  echo "$env $(grep -c debug_fin gpurun_out/stress_${T}.txt) debug lines $(tail -1 gpurun_out/stress_${T}.txt | cut -c1-100)"
done
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_small.py \
  > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs > gpurun_out/ab_${T}.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
k = {x["name"]: x for x in d["kernels"]}
g = lambda n: round(k[n]["total_ms"] / max(1, k[n]["launches"]) * 1e3, 1) if n in k else None
print(round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share", round(d["kernel_share_of_step"], 3),
      "entry->first", g("host:entry->first_launch"), "prep", g("host:first:prepare+alloc"), "c+p", g("host:complete+plan"),
      "complete", g("host:complete"), "wait_fast", g("host:wait_fast"))
PY
done
CSM_LIB=roborts-edu-slam_amd/lib/libroborts_csm-btrace.so timeout -k 10 200 python tools/box_trace.py > gpurun_out/box_trace_${T}.json \
  2> gpurun_out/box_trace_${T}.err || { tail -5 gpurun_out/box_trace_${T}.err; exit 1; }
cat gpurun_out/box_trace_${T}.json
