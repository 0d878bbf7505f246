#!/bin/bash
# r04: progressive first-level spans (CSM_FIRST_WINDOWS / CSM_SPAN_GROWTH): the driver's parity
# tests, then A/B of the config-2 line against the old two-span form.
set -o pipefail
mkdir -p gpurun_out
T=${1:-s8}
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "split or pipelined or host_signal or three_level or dead" > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || exit $rc
for env in "X=0" "CSM_FIRST_WINDOWS=64 CSM_SPAN_GROWTH=100000" "CSM_FIRST_WINDOWS=64" "CSM_SPAN_GROWTH=2" "X=0" "CSM_FIRST_WINDOWS=64 CSM_SPAN_GROWTH=100000"; do
  env $env timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs > gpurun_out/ab_${T}.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}.json "$env" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
k = {x["name"]: x for x in d["kernels"]}
e = k.get("host:entry->first_launch", {"total_ms": 0, "launches": 1})
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share",
      round(d["kernel_share_of_step"], 3), "entry->first", round(e["total_ms"] / max(1, e["launches"]) * 1e3, 1), "us")
PY
done
