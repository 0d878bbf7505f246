#!/bin/bash
# r04: box kernels, isolated timing (tools/box_kbench.py: coarse level only, unpipelined) after the
# palette/parity GPU tests of the v11 pair kernel. pdiag1: no accumulation (wrong scores, timing only).
set -o pipefail
mkdir -p gpurun_out
T=${1:-pal3}
out=gpurun_out/kbench_${T}.txt
: > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_palette.py \
  tests/test_gpu_parity.py -k "palette or box or headline or phase or variants" > gpurun_out/pytest_${T}.log 2>&1 || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -2 gpurun_out/pytest_${T}.log
timeout -k 10 120 tools/ubench/ta_probe > gpurun_out/ta_probe_${T}.txt 2>&1 || exit $?
for env in "CSM_BOX_PALETTE=0" "CSM_BOX_PAIR=0" "CSM_BOX_PAIR=1" "CSM_BOX_PAIR=0 CSM_LIB=roborts-edu-slam_amd/lib/libroborts_csm-pdiag1.so" "CSM_BOX_PAIR=1 CSM_LIB=roborts-edu-slam_amd/lib/libroborts_csm-pdiag1.so"; do
  echo "# $env" >> $out
  env $env timeout -k 10 200 python tools/box_kbench.py >> $out 2>&1 || exit $?
done
for st in 0 1; do echo "# CSM_PHASE_STRIPS=$st" >> $out; CSM_PHASE_STRIPS=$st timeout -k 10 200 python tools/box_kbench.py --level 1 >> $out 2>&1 || exit $?; done
timeout -k 10 200 python tools/box_kbench.py --level 2 >> $out 2>&1 || exit $?
grep '^[{#]' $out
