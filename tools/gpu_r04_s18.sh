#!/bin/bash
# r04: exact pass on CUs of its own (CSM_EXACT_CUS) vs shared CUs
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-s18}
CSM_EXACT_CUS=8 timeout -k 10 200 python tools/stress_ties.py --iters 20 > gpurun_out/stress_${T}.txt 2>&1 || { tail -5 gpurun_out/stress_${T}.txt; exit 1; }
echo "stress (8 CUs): $(tail -1 gpurun_out/stress_${T}.txt | cut -c1-90)"
: > gpurun_out/ab_${T}.txt
for rep in 1 2; do
  for n in 0 8 16; do
    env $( [ $n = 0 ] || echo CSM_EXACT_CUS=$n ) timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-latency --no-host-inputs \
      > gpurun_out/ab_${T}.json 2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
    python3 - gpurun_out/ab_${T}.json "exact_cus=$n" <<'PY' | tee -a gpurun_out/ab_${T}.txt
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share", round(d["kernel_share_of_step"], 4),
      "exact", round(d["exact_finish_side_stream_ms_per_step"], 4), "pair", round(d["roofline"]["avg_launch_ms"], 4))
PY
  done
done
rm -rf gpurun_out/prof_${T}
CSM_EXACT_CUS=8 CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-latency --no-b109 --no-lc-leg --no-host-inputs > gpurun_out/prof_${T}.json 2> gpurun_out/prof_${T}.err \
  || { tail -20 gpurun_out/prof_${T}.err; exit 1; }
f=$(find gpurun_out/prof_${T} -name '*kernel_trace.csv' | head -1)
python3 tools/dispatch_stats.py "$f" score_ finish_ > gpurun_out/dispatch_${T}.json
python3 -c "import json,sys; [print(k, {x: d[x] for x in ('launches','p50_us','p99_us','max_us')}) for k, d in json.load(open(sys.argv[1])).items()]" gpurun_out/dispatch_${T}.json
