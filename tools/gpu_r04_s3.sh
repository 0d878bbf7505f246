#!/bin/bash
# r04: stress of the 3-value-map driver under its knobs, the default config-2 bench line, the
# online line (latency tail attribution), then the exact-pass priority A/B under rocprof.
set -o pipefail
mkdir -p gpurun_out
T=${1:-s3}
for env in "X=0" "CSM_EARLY_COMPLETE=0" "CSM_HOST_SIGNAL=0" "CSM_FIRST_WINDOWS=0" "CSM_EXACT_STREAM=0"; do
  env $env timeout -k 10 200 python tools/stress_ties.py --iters 40 >> gpurun_out/stress_${T}.txt 2>&1 || { tail -5 gpurun_out/stress_${T}.txt; exit 1; }
done
cut -c1-600 gpurun_out/stress_${T}.txt
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err \
  || { tail -20 gpurun_out/bench_${T}.err; exit 1; }
python3 - gpurun_out/bench_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step finish", round(d["finish_ms_per_step"], 3),
      "share", round(d["kernel_share_of_step"], 3), "host_inputs", json.dumps(d.get("value_host_inputs"))[:300])
for k in d["kernels"]:
    if k["name"].startswith(("score_", "finish_kernel")):
        print(" ", k["name"], k["launches"], round(k["total_ms"] / k["launches"], 4))
PY
timeout -k 10 300 python bench.py --workload online --steps 400 --warmup 20 > gpurun_out/online_${T}.json \
  2> gpurun_out/online_${T}.err || { tail -20 gpurun_out/online_${T}.err; exit 1; }
python3 - gpurun_out/online_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
c = d["config"]
print("online", round(d["value"], 1), "scans/s", c["latency_ms"])
print(json.dumps(c["latency_tail"])[:3000])
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 0 1; do
  rm -rf gpurun_out/prof_${T}_p$p
  CSM_EXACT_PRIO=$p CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_p$p \
    -o run --output-format csv -- python3 bench.py --no-cpu --no-latency --no-b109 --no-lc-leg --no-host-inputs \
    > gpurun_out/prof_${T}_p$p.json 2> gpurun_out/prof_${T}_p$p.err || { tail -20 gpurun_out/prof_${T}_p$p.err; exit 1; }
  f=$(find gpurun_out/prof_${T}_p$p -name '*kernel_trace.csv' | head -1)
  echo "# CSM_EXACT_PRIO=$p"
  python3 tools/dispatch_stats.py "$f" score_ finish_ > gpurun_out/dispatch_${T}_p$p.json && cat gpurun_out/dispatch_${T}_p$p.json
  python3 - gpurun_out/prof_${T}_p$p.json $p <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print("prio", sys.argv[2], "under rocprof", round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step")
PY
done
