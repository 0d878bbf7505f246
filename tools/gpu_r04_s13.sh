#!/bin/bash
# r04: submitted batches (csm_scan_matchers_submit) and the split hand-off: the whole GPU suite, smoke,
# config-2 lines submitted vs one call per step, a kernel trace of the submitted form, the online line.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-s13}
timeout -k 10 200 python tools/stress_ties.py --iters 40 > gpurun_out/stress_${T}.txt 2>&1 || { tail -5 gpurun_out/stress_${T}.txt; exit 1; }
echo "stress: $(tail -1 gpurun_out/stress_${T}.txt | cut -c1-90)"
CSM_FINISH_SIDE=1 timeout -k 10 200 python tools/stress_ties.py --iters 20 > gpurun_out/stress_${T}_side.txt 2>&1 || { tail -5 gpurun_out/stress_${T}_side.txt; exit 1; }
echo "stress (side kernel): $(tail -1 gpurun_out/stress_${T}_side.txt | cut -c1-90)"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 || { cat gpurun_out/smoke_${T}.log; exit 1; }
tail -1 gpurun_out/smoke_${T}.log
for mode in "0 " "0 --sync-steps" "1 " "0 " "0 --sync-steps" "1 "; do
  side=${mode%% *}; flag=${mode#* }
  CSM_FINISH_SIDE=$side timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs $flag > gpurun_out/ab_${T}.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}.json "side=$side ${flag:-submitted}" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
ks = ("kernel_stream_ms_per_step", "exact_finish_side_stream_ms_per_step", "kernel_share_of_step")
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step", {k: round(d[k], 4) for k in ks if d.get(k) is not None})
PY
done
rm -rf gpurun_out/prof_${T}
CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-latency --no-b109 --no-lc-leg --no-host-inputs > gpurun_out/prof_${T}.json 2> gpurun_out/prof_${T}.err \
  || { tail -20 gpurun_out/prof_${T}.err; exit 1; }
f=$(find gpurun_out/prof_${T} -name '*kernel_trace.csv' | head -1)
python3 tools/timeline_gaps.py "$f" 20 | head -20
python3 tools/dispatch_stats.py "$f" score_ finish_ > gpurun_out/dispatch_${T}.json
rm -rf gpurun_out/prof_${T}_side
CSM_FINISH_SIDE=1 CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_side -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-latency --no-b109 --no-lc-leg --no-host-inputs > gpurun_out/prof_${T}_side.json 2> gpurun_out/prof_${T}_side.err \
  || { tail -20 gpurun_out/prof_${T}_side.err; exit 1; }
f=$(find gpurun_out/prof_${T}_side -name '*kernel_trace.csv' | head -1)
python3 tools/dispatch_stats.py "$f" score_ finish_ > gpurun_out/dispatch_${T}_side.json
python3 -c "import json,sys; [print(k, {x: d[x] for x in ('launches','p50_us','p99_us','max_us')}) for f in sys.argv[1:] for k, d in json.load(open(f)).items() if k.startswith('finish_') and 'fast' not in k]" gpurun_out/dispatch_${T}.json gpurun_out/dispatch_${T}_side.json
timeout -k 10 300 python bench.py --workload online --steps 400 --warmup 20 > gpurun_out/online_${T}.json \
  2> gpurun_out/online_${T}.err || { tail -20 gpurun_out/online_${T}.err; exit 1; }
python3 - gpurun_out/online_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
c = d["config"]; l = c["latency_ms"]
print("online", round(d["value"], 1), "scans/s p50 %.3f p99 %.3f" % (l["p50"], l["p99"]))
PY
