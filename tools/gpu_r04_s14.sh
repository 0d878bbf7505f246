#!/bin/bash
# r04: the deferred last hand-off of submitted batches (CSM_DEFER_HANDOFF): GPU suite, smoke, stress,
# config-2 A/B (deferred / not deferred / one call per step).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-s14}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 || { cat gpurun_out/smoke_${T}.log; exit 1; }
tail -1 gpurun_out/smoke_${T}.log
timeout -k 10 200 python tools/stress_ties.py --iters 40 > gpurun_out/stress_${T}.txt 2>&1 || { tail -5 gpurun_out/stress_${T}.txt; exit 1; }
echo "stress: $(tail -1 gpurun_out/stress_${T}.txt | cut -c1-90)"
for mode in "1 " "0 " "1 --sync-steps" "1 " "0 " "1 --sync-steps"; do
  d=${mode%% *}; flag=${mode#* }
  CSM_DEFER_HANDOFF=$d timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-latency $flag > gpurun_out/ab_${T}.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}.json "defer=$d ${flag:-submitted}" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
ks = ("kernel_stream_ms_per_step", "exact_finish_side_stream_ms_per_step", "kernel_share_of_step")
h = d.get("value_host_inputs") or {}
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step", {k: round(d[k], 4) for k in ks if d.get(k) is not None},
      "host_inputs", round(h.get("value", 0) / 1e9, 3), h.get("same_result_as_resident"))
PY
done
rm -rf gpurun_out/prof_${T}
CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-latency --no-b109 --no-lc-leg --no-host-inputs > gpurun_out/prof_${T}.json 2> gpurun_out/prof_${T}.err \
  || { tail -20 gpurun_out/prof_${T}.err; exit 1; }
f=$(find gpurun_out/prof_${T} -name '*kernel_trace.csv' | head -1)
python3 tools/timeline_gaps.py "$f" 20 | head -20
