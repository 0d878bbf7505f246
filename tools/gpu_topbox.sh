# Beam-box top level: search tests, then the loop-closure and willow benches
# (int16 box copy, then CSM_TOPBOX_ELEM=4: the int32 copy) and a kernel-trace
# summary of the loop-closure bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_topbox.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_topbox.log
[ $rc -eq 0 ] || exit $rc
for e in 2 4; do
  CSM_TOPBOX_ELEM=$e timeout -k 10 300 python bench.py --workload loop_closure --steps 5 --warmup 2 --no-cpu > gpurun_out/lc_topbox$e.json 2> gpurun_out/lc_topbox$e.err || exit $?
  CSM_TOPBOX_ELEM=$e timeout -k 10 300 python bench.py --workload willow --steps 5 --warmup 1 --no-cpu > gpurun_out/willow_topbox$e.json 2> gpurun_out/willow_topbox$e.err || exit $?
  echo "elem $e done"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lc_topbox -o run --output-format csv -- python3 bench.py --workload loop_closure --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_lc_topbox.json 2> gpurun_out/prof_lc_topbox.err || exit $?
echo "prof done"
