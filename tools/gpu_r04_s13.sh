#!/bin/bash
# r04: submitted batches (csm_scan_matchers_submit) and the split hand-off: the whole GPU suite, smoke,
# config-2 lines submitted vs one call per step, a kernel trace of the submitted form, the online line.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-s13}
timeout -k 10 200 python tools/stress_ties.py --iters 40 > gpurun_out/stress_${T}.txt 2>&1 || { tail -5 gpurun_out/stress_${T}.txt; exit 1; }
echo "stress: $(tail -1 gpurun_out/stress_${T}.txt | cut -c1-90)"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 || { cat gpurun_out/smoke_${T}.log; exit 1; }
tail -1 gpurun_out/smoke_${T}.log
for mode in "" "--sync-steps" "" "--sync-steps"; do
  timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs $mode > gpurun_out/ab_${T}.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}.json "${mode:-submitted}" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share", round(d["kernel_share_of_step"], 3))
PY
done
rm -rf gpurun_out/prof_${T}
CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-latency --no-b109 --no-lc-leg --no-host-inputs > gpurun_out/prof_${T}.json 2> gpurun_out/prof_${T}.err \
  || { tail -20 gpurun_out/prof_${T}.err; exit 1; }
f=$(find gpurun_out/prof_${T} -name '*kernel_trace.csv' | head -1)
python3 tools/timeline_gaps.py "$f" 20 | head -20
python3 tools/dispatch_stats.py "$f" score_ finish_ > gpurun_out/dispatch_${T}.json
timeout -k 10 300 python bench.py --workload online --steps 400 --warmup 20 > gpurun_out/online_${T}.json \
  2> gpurun_out/online_${T}.err || { tail -20 gpurun_out/online_${T}.err; exit 1; }
python3 - gpurun_out/online_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
c = d["config"]; l = c["latency_ms"]
print("online", round(d["value"], 1), "scans/s p50 %.3f p99 %.3f" % (l["p50"], l["p99"]))
PY
