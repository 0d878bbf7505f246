#!/bin/bash
# r04: uneven part split A/B (CSM_PART0_PERMILLE), then the online line with the per-map update times.
set -o pipefail
mkdir -p gpurun_out
T=${1:-s12}
for pm in 500 600 550 650 500 600 550 650; do
  CSM_PART0_PERMILLE=$pm timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs > gpurun_out/ab_${T}.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}.json $pm <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share", round(d["kernel_share_of_step"], 3))
PY
done
timeout -k 10 300 python bench.py --workload online --steps 400 --warmup 20 > gpurun_out/online_${T}.json \
  2> gpurun_out/online_${T}.err || { tail -20 gpurun_out/online_${T}.err; exit 1; }
python3 - gpurun_out/online_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
c = d["config"]
print("online", round(d["value"], 1), "scans/s", c["latency_ms"])
t = c["latency_tail"]
print(json.dumps(t["phase_ms"]))
for s in t["slowest"]:
    print(s["scan"], round(s["ms"], 3), s["kept"], s["fine_map_grew"], s["phases_ms"], s["outside_call_ms"])
PY
