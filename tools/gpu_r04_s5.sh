#!/bin/bash
# r04: the early-completion mismatch caught in the act (CSM_DEBUG_FIN: the last level's FinishOut as
# completed vs what the finish left once the device is idle).
set -o pipefail
mkdir -p gpurun_out
T=${1:-s5}
for pr in 0 1; do
  CSM_DEBUG_FIN=1 timeout -k 10 200 python tools/stress_ties.py --iters 60 --profiling $pr > gpurun_out/stress_${T}_p$pr.txt 2>&1 \
    || { tail -5 gpurun_out/stress_${T}_p$pr.txt; exit 1; }
  echo "profiling=$pr $(grep -c 'debug_fin' gpurun_out/stress_${T}_p$pr.txt) debug lines; $(tail -1 gpurun_out/stress_${T}_p$pr.txt | cut -c1-150)"
  grep 'debug_fin' gpurun_out/stress_${T}_p$pr.txt | head -12 || true
done
