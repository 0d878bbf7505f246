#!/bin/bash
# r04: submitted-batch part split and split hand-off around the final defaults (env knobs only)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-s17}
: > gpurun_out/sweep_${T}.txt
for rep in 1 2; do
  for cfg in "500 1" "450 1" "500 0" "550 1" "400 1"; do
    set -- $cfg
    CSM_PART0_PERMILLE_SUBMIT=$1 CSM_SPLIT_HANDOFF=$2 timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-latency --no-host-inputs \
      > gpurun_out/sw_${T}.json 2> gpurun_out/sw_${T}.err || { tail -20 gpurun_out/sw_${T}.err; exit 1; }
    python3 - gpurun_out/sw_${T}.json "permille=$1 split=$2" <<'PY' | tee -a gpurun_out/sweep_${T}.txt
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share", round(d["kernel_share_of_step"], 4))
PY
  done
done
