set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_search1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_search1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for d in -1 4 5; do
  timeout -k 10 200 python bench.py --workload loop_closure --steps 3 --warmup 1 --no-cpu --depth $d > gpurun_out/lc_d$d.json 2> gpurun_out/lc_d$d.err || exit $?
  echo "lc depth $d done"
done
for d in -1 4 5; do
  timeout -k 10 200 python bench.py --workload willow --steps 5 --warmup 1 --no-cpu --depth $d > gpurun_out/willow_d$d.json 2> gpurun_out/willow_d$d.err || exit $?
  echo "willow depth $d done"
done
exit $rc
