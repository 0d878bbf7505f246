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
out=gpurun_out/kbench_${T}.txt; : > $out
for lib in "" roborts-edu-slam_amd/lib/libroborts_csm-pf6.so roborts-edu-slam_amd/lib/libroborts_csm-pf8.so ""; do
  echo "# lib=$lib" >> $out; CSM_LIB=$lib timeout -k 10 200 python tools/box_kbench.py >> $out 2>&1 || exit $?
done
grep '^[{#]' $out | cut -c1-200
timeout -k 10 200 python tools/stress_ties.py --iters 40 > gpurun_out/stress_${T}.txt 2>&1 || { tail -5 gpurun_out/stress_${T}.txt; exit 1; }
echo "stress (split hand-off from 8 windows): $(tail -1 gpurun_out/stress_${T}.txt | cut -c1-90)"
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || exit $rc
for sp in 1 0 1 0; do
  CSM_SPLIT_HANDOFF=$sp timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs > gpurun_out/ab_${T}.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}.json $sp <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print("split_handoff", sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share", round(d["kernel_share_of_step"], 3))
PY
done
