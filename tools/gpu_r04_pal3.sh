#!/bin/bash
# r04: palette kernel timing by phase (pdiag1: no accumulation, pdiag2: + no cell-by-cell pass,
# pdiag3: + no run lists) — wrong scores, timing only.
set -o pipefail
mkdir -p gpurun_out
T=${1:-pal3}
for v in "" pdiag1 pdiag2 pdiag3; do
  lib=""; [ -n "$v" ] && lib=roborts-edu-slam_amd/lib/libroborts_csm-$v.so
  CSM_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs --steps 20 --warmup 10 > gpurun_out/bench_${T}_${v:-default}.json 2>&1 || exit $?
  python3 - gpurun_out/bench_${T}_${v:-default}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(sys.argv[1], round(d["ms_per_step"], 4), "ms/step",
      [(k["name"], round(k["total_ms"] / k["launches"], 4)) for k in d["kernels"] if k["name"].startswith("score_box")])
PY
done
