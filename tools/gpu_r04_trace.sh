#!/bin/bash
# r04: the pair box kernel's phase stamps (CSM_BOX_TRACE build), then the config-2 bench on the
# default build (no CPU / loop-closure / B=109 / host-input legs).
set -o pipefail
mkdir -p gpurun_out
T=${1:-tr1}
CSM_LIB=roborts-edu-slam_amd/lib/libroborts_csm-btrace.so timeout -k 10 200 python tools/box_trace.py \
  > gpurun_out/box_trace_${T}.json 2> gpurun_out/box_trace_${T}.err || { tail -20 gpurun_out/box_trace_${T}.err; exit 1; }
cat gpurun_out/box_trace_${T}.json
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
