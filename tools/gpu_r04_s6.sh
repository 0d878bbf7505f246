#!/bin/bash
# r04: the sealed FinishOut: stress (with the debug snapshot), the GPU suite, smoke, the config-2 line.
set -o pipefail
mkdir -p gpurun_out
T=${1:-s6}
for pr in 0 1; do
  CSM_DEBUG_FIN=1 timeout -k 10 200 python tools/stress_ties.py --iters 60 --profiling $pr > gpurun_out/stress_${T}_p$pr.txt 2>&1 \
    || { tail -5 gpurun_out/stress_${T}_p$pr.txt; exit 1; }
  echo "profiling=$pr $(grep -c 'debug_fin' gpurun_out/stress_${T}_p$pr.txt) debug lines; $(tail -1 gpurun_out/stress_${T}_p$pr.txt | cut -c1-150)"
done
CSM_FIRST_WINDOWS=0 timeout -k 10 200 python tools/stress_ties.py --iters 60 > gpurun_out/stress_${T}_fw0.txt 2>&1 || exit $?
echo "first_windows=0 $(tail -1 gpurun_out/stress_${T}_fw0.txt | cut -c1-120)"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 || { cat gpurun_out/smoke_${T}.log; exit 1; }
tail -1 gpurun_out/smoke_${T}.log
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err || { tail -20 gpurun_out/bench_${T}.err; exit 1; }
python3 - gpurun_out/bench_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step finish", round(d["finish_ms_per_step"], 3),
      "share", round(d["kernel_share_of_step"], 3), "host_inputs", round(d["value_host_inputs"]["value"] / 1e9, 3))
PY
