#!/bin/bash
# r04: palette kernel timing split (run lists only: the pdiag1 build) and its PMC counters.
set -o pipefail
mkdir -p gpurun_out
T=${1:-pal2}
for lib in "" roborts-edu-slam_amd/lib/libroborts_csm-pdiag1.so grouped; do
  pal=1; if [ "$lib" = grouped ]; then pal=0; lib=""; fi
  CSM_BOX_PALETTE=$pal CSM_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 > gpurun_out/bench_${T}_$(basename "${lib:-default}")_$pal.json 2>&1 || exit $?
  python3 - gpurun_out/bench_${T}_$(basename "${lib:-default}")_$pal.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(sys.argv[1], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step",
      [(k["name"], round(k["total_ms"] / k["launches"], 4)) for k in d["kernels"] if k["name"].startswith("score_")])
PY
done
timeout -k 10 900 tools/pmc_roofline.sh gpurun_out/pmc_$T || exit $?
cat gpurun_out/pmc_$T/summary.txt | head -60
