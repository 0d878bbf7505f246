#!/bin/bash
# r04: driver A/B (parts in flight, first-span windows) on the sealed build, then the PMC passes
# of the config-2 kernels for the roofline (profiles/r04/counters.json).
set -o pipefail
mkdir -p gpurun_out
T=${1:-s7}
for env in "X=0" "CSM_PIPELINE_PARTS=3" "CSM_PIPELINE_PARTS=4" "CSM_FIRST_WINDOWS=256" "CSM_FIRST_WINDOWS=16" "X=0"; do
  env $env timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-host-inputs > gpurun_out/ab_${T}.json \
    2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
  python3 - gpurun_out/ab_${T}.json "$env" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share", round(d["kernel_share_of_step"], 3))
PY
done
bash tools/pmc_roofline.sh gpurun_out/pmc_${T} || exit $?
tail -30 gpurun_out/pmc_${T}/summary.txt
