#!/bin/bash
# r04: host-signal diagnostic, palette box kernel parity, palette A/B on config 2.
set -o pipefail
mkdir -p gpurun_out
T=${1:-pal}
timeout -k 10 300 python -u tools/diag_host_signal.py 150 > gpurun_out/diag_hs_$T.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/diag_host_signal.py 150 CSM_EARLY_COMPLETE=0 >> gpurun_out/diag_hs_$T.txt 2>&1 || exit $?
tail -4 gpurun_out/diag_hs_$T.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_gpu_palette.py \
  "tests/test_gpu_parity.py::test_box_kernel_edge_beams" "tests/test_gpu_parity.py::test_headline_runs_row_segment_kernels" \
  > gpurun_out/pytest_$T.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$T.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in 1 0 1 0; do
  CSM_BOX_PALETTE=$m timeout -k 10 300 python bench.py --no-cpu --no-lc-leg --no-b109 > gpurun_out/bench_${T}_pal$m.json 2> gpurun_out/bench_${T}_pal$m.err || exit $?
  python3 - gpurun_out/bench_${T}_pal$m.json $m <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
rl = d["roofline"]
print("palette", sys.argv[2], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step", rl["kernel"], round(rl["avg_launch_ms"], 4))
PY
done
exit $rc
