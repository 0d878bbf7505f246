#!/bin/bash
# r04: 16 strip copies by default, sealed copies of only the listed pieces: stress, the GPU suite,
# repeated config-2 lines with the host's first-launch phases.
set -o pipefail
mkdir -p gpurun_out
T=${1:-s11}
CSM_DEBUG_FIN=1 timeout -k 10 200 python tools/stress_ties.py --iters 40 > gpurun_out/stress_${T}.txt 2>&1 || { tail -5 gpurun_out/stress_${T}.txt; exit 1; }
echo "$(grep -c debug_fin gpurun_out/stress_${T}.txt) debug lines $(tail -1 gpurun_out/stress_${T}.txt | cut -c1-100)"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs > gpurun_out/ab_${T}_$i.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}_$i.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
k = {x["name"]: x for x in d["kernels"]}
g = lambda n: round(k[n]["total_ms"] / max(1, k[n]["launches"]) * 1e3, 1) if n in k else None
print(round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share", round(d["kernel_share_of_step"], 3),
      "e->split", g("host:first:entry->split"), "prep", g("host:first:prepare"), "prep+alloc", g("host:first:prepare+alloc"),
      "plan", g("host:first:plan"), "e->first", g("host:entry->first_launch"), "c+p", g("host:complete+plan"),
      "complete", g("host:complete"), "between", g("host:between_calls"))
PY
done
