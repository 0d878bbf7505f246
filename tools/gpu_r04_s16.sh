#!/bin/bash
# r04: submitted-batch defaults (one first launch, 50/50 parts) against the earlier ones
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-s16}
: > gpurun_out/ab_${T}.txt
for rep in 1 2; do
  for cfg in "default" "CSM_FIRST_WINDOWS_SUBMIT=128 CSM_PART0_PERMILLE_SUBMIT=550"; do
    env $( [ "$cfg" = default ] || echo $cfg ) timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 --no-latency --no-host-inputs \
      > gpurun_out/ab_${T}.json 2> gpurun_out/ab_${T}.err || { tail -20 gpurun_out/ab_${T}.err; exit 1; }
    python3 - gpurun_out/ab_${T}.json "$cfg" <<'PY' | tee -a gpurun_out/ab_${T}.txt
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step share", round(d["kernel_share_of_step"], 4),
      "pair", round(d["roofline"]["avg_launch_ms"], 4))
PY
  done
done
