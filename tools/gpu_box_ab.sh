#!/bin/bash
# Box-kernel A/B on one GPU: the GPU suite on the default build, the parity
# tests under each alternative box mode, then interleaved config-2 benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_box.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_box.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in g2 g1; do
  CSM_BOX=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_box_$m.log 2>&1 || { echo "parity $m failed"; tail -5 gpurun_out/pytest_box_$m.log; exit 1; }
  echo "parity $m ok"
done
for i in 1 2; do
  for m in default g2 g1 runs; do
    if [ $m = default ]; then e=""; else e="CSM_BOX=$m"; fi
    env $e timeout -k 10 200 python bench.py --no-cpu --no-b109 > gpurun_out/bench_box_${m}_$i.json 2> gpurun_out/bench_box_${m}_$i.err || exit $?
  done
done
exit 0
