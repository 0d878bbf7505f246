#!/bin/bash
# r04: bisect test_host_signal_split_levels_with_ties (3-value map) over the r04 kernel knobs,
# then the rest of the GPU suite and the isolated box-kernel timings.
set -o pipefail
mkdir -p gpurun_out
T=${1:-bis}
K=tests/test_gpu_parity.py::test_host_signal_split_levels_with_ties
for env in "X=0" "CSM_BOX_PAIR=0" "CSM_BOX_PALETTE=0" "CSM_PHASE_STRIPS=0" "CSM_EARLY_COMPLETE=0" "CSM_FINISH=exact"; do
  env $env timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread $K > gpurun_out/bis_${T}.log 2>&1
  rc=$?
  echo "$env rc=$rc $(tail -1 gpurun_out/bis_${T}.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect $K \
  > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
out=gpurun_out/kbench_${T}.txt
: > $out
for env in "CSM_BOX_PAIR=1" "CSM_BOX_PAIR=0" "CSM_BOX_PALETTE=0"; do
  echo "# $env" >> $out
  env $env timeout -k 10 200 python tools/box_kbench.py >> $out 2>&1 || exit $?
done
for l in 1 2; do echo "# level $l" >> $out; timeout -k 10 200 python tools/box_kbench.py --level $l >> $out 2>&1 || exit $?; done
grep '^[{#]' $out
