# Loop-closure and willow legs on the final build: PMC passes over the
# loop-closure bench (counters for its top-level kernel), then both legs with
# their CPU baselines and rooflines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_lc_final.log 2>&1 || { tail -5 gpurun_out/pytest_lc_final.log; exit 1; }
bash tools/pmc_roofline.sh gpurun_out/pmclc --workload loop_closure --steps 2 --warmup 1 --no-cpu || exit $?
cp gpurun_out/pmclc/counters.json profiles/r02/counters_lc.json
timeout -k 10 300 python bench.py --workload loop_closure --steps 5 --warmup 2 > gpurun_out/lc_final.json 2> gpurun_out/lc_final.err || exit $?
timeout -k 10 300 python bench.py --workload willow --steps 5 --warmup 1 > gpurun_out/willow_final.json 2> gpurun_out/willow_final.err || exit $?
echo "lc final done"
