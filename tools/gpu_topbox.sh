# Pyramid search: the search tests, the loop-closure and willow benches and a
# kernel-trace summary of the loop-closure bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_topbox.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_topbox.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload loop_closure --steps 5 --warmup 2 --no-cpu > gpurun_out/lc_topbox2.json 2> gpurun_out/lc_topbox2.err || exit $?
timeout -k 10 300 python bench.py --workload willow --steps 5 --warmup 1 --no-cpu > gpurun_out/willow_topbox2.json 2> gpurun_out/willow_topbox2.err || exit $?
echo "benches done"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_lc_topbox
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lc_topbox -o run --output-format csv -- python3 bench.py --workload loop_closure --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_lc_topbox.json 2> gpurun_out/prof_lc_topbox.err || exit $?
echo "prof done"
