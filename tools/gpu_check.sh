#!/bin/bash
# One GPU call: the GPU test suite, then (only if no test crashed the process)
# the given follow-up steps. Test failures (pytest rc 1) do not stop the
# follow-ups; a crash, abort or time limit does.
#   tools/gpu_check.sh TAG [step ...]   steps: smoke, stress, pmc, adapter, bench, b109, online, lc, willow, prof
# (TESTS=0: no test suite; TESTS="-k expr" selects tests)
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
rc=0
if [ "${TESTS:-}" != "0" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTS:-} \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for step in "$@"; do
  case $step in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
             > gpurun_out/smoke_$TAG.log 2>&1 || exit $? ;;
    stress) timeout -k 10 300 python tools/stress_ties.py --iters 60 > gpurun_out/stress_$TAG.json 2>&1 || exit $? ;;
    b109) timeout -k 10 300 python bench.py --levels sim --no-cpu --no-lc-leg --no-host-inputs \
            > gpurun_out/b109_$TAG.json 2> gpurun_out/b109_$TAG.err || exit $? ;;
    online) timeout -k 10 300 python bench.py --workload online --steps 400 \
            > gpurun_out/online_$TAG.json 2> gpurun_out/online_$TAG.err || exit $? ;;
    pmc) timeout -k 10 900 tools/pmc_roofline.sh gpurun_out/pmc_$TAG || exit $? ;;
    adapter) timeout -k 10 300 tests/cpp/build/adapter_run bench 40 3000 > gpurun_out/adapter_$TAG.json || exit $? ;;
    bench) timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $? ;;
    lc) timeout -k 10 300 python bench.py --workload loop_closure --steps 3 --warmup 1 \
          > gpurun_out/lc_$TAG.json 2> gpurun_out/lc_$TAG.err || exit $? ;;
    willow) timeout -k 10 300 python bench.py --workload willow --steps 5 --warmup 1 \
          > gpurun_out/willow_$TAG.json 2> gpurun_out/willow_$TAG.err || exit $? ;;
    prof) (cd /tmp && export TMPDIR=/tmp; true); export TMPDIR=/tmp
          timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- \
            python3 bench.py --no-cpu --no-latency --no-b109 --no-lc-leg > gpurun_out/prof_bench_$TAG.json 2>&1 || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step done"
done
exit $rc
