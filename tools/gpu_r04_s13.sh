#!/bin/bash
# r04: the online line's latency tail under host-side variants (eager code-object loading, CPU pinning,
# fewer pool threads).
set -o pipefail
mkdir -p gpurun_out
T=${1:-s13}
run() {  # run LABEL CMD...
  local lab=$1; shift
  timeout -k 10 300 "$@" python bench.py --workload online --steps 400 --warmup 20 --no-cpu > gpurun_out/online_${T}.json \
    2> gpurun_out/online_${T}.err || { tail -20 gpurun_out/online_${T}.err; exit 1; }
  python3 - gpurun_out/online_${T}.json "$lab" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
c = d["config"]; t = c["latency_tail"]; l = c["latency_ms"]
print(sys.argv[2], "p50 %.3f p99 %.3f max %.3f" % (l["p50"], l["p99"], l["max"]), "slowest:",
      [(s["scan"], round(s["ms"], 2), round(s["phases_ms"]["match"], 2), round(s["phases_ms"]["update_map"], 2)) for s in t["slowest"][:5]])
PY
}
run default env
# (HIP_ENABLE_DEFERRED_LOADING=0 segfaulted at load on the box, r04)
run pinned taskset -c 8-23
run threads4 env CSM_HOST_THREADS=4
run default2 env
