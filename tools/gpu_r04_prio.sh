#!/bin/bash
# r04: the exact finish pass's dispatch-time tail under rocprofv3 kernel traces, with the
# exact pass's stream at normal and at the highest priority (CSM_EXACT_PRIO), then the
# config-2 bench both ways. Whole level-parts per dispatch (CSM_FIRST_WINDOWS=0).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-prio}
for p in 0 1; do
  rm -rf gpurun_out/prof_${T}_p$p
  CSM_EXACT_PRIO=$p CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_p$p \
    -o run --output-format csv -- python3 bench.py --no-cpu --no-latency --no-b109 --no-lc-leg --no-host-inputs \
    > gpurun_out/prof_${T}_p$p.json 2> gpurun_out/prof_${T}_p$p.err || { tail -20 gpurun_out/prof_${T}_p$p.err; exit 1; }
  f=$(ls gpurun_out/prof_${T}_p$p/*/*/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(find gpurun_out/prof_${T}_p$p -name '*kernel_trace.csv' | head -1)
  echo "# CSM_EXACT_PRIO=$p"
  python3 tools/dispatch_stats.py "$f" score_ finish_ > gpurun_out/dispatch_${T}_p$p.json && cat gpurun_out/dispatch_${T}_p$p.json
done
for p in 0 1 0 1; do
  CSM_EXACT_PRIO=$p timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs \
    > gpurun_out/bench_${T}_p$p.json 2> gpurun_out/bench_${T}_p$p.err || { tail -20 gpurun_out/bench_${T}_p$p.err; exit 1; }
  python3 - gpurun_out/bench_${T}_p$p.json $p <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print("prio", sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step exact",
      round(d["exact_finish_side_stream_ms_per_step"], 3), "finish", round(d["finish_ms_per_step"], 3))
PY
done
