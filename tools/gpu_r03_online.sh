# r03: config 5 lines (online alone, 40 Hz with the back end attached) and
# the drop-in adapter, PMC counters of the few-window path, kernel traces.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
if [ "${PMC:-1}" = 1 ]; then
  bash tools/pmc_roofline.sh gpurun_out/pmc_small_$TAG --workload online --steps 100 --warmup 10 --no-cpu || exit $?
  mkdir -p profiles/r03 && cp gpurun_out/pmc_small_$TAG/counters.json profiles/r03/counters_small.json
  echo "pmc done"
fi
timeout -k 10 300 python bench.py --workload online --steps 300 --warmup 20 > gpurun_out/online_$TAG.json 2> gpurun_out/online_$TAG.err || exit $?
echo "online done"
timeout -k 10 300 python bench.py --workload online --attach-backend --rate-hz 40 --steps 300 --warmup 20 > gpurun_out/online_be40_$TAG.json 2> gpurun_out/online_be40_$TAG.err || exit $?
echo "online+backend 40 Hz done"
timeout -k 10 300 python bench.py --workload online --attach-backend --steps 300 --warmup 20 --no-cpu > gpurun_out/online_be_unpaced_$TAG.json 2> gpurun_out/online_be_unpaced_$TAG.err || exit $?
echo "online+backend unpaced done"
timeout -k 10 300 python bench.py --workload adapter --steps 40 > gpurun_out/adapter_$TAG.json 2> gpurun_out/adapter_$TAG.err || exit $?
echo "adapter done"
if [ "${TRACE:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_online_$TAG -o run --output-format csv -- python3 bench.py --workload online --steps 200 --warmup 20 --no-cpu > gpurun_out/prof_online_$TAG.json 2> gpurun_out/prof_online_$TAG.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_online_be_$TAG -o run --output-format csv -- python3 bench.py --workload online --attach-backend --rate-hz 40 --steps 200 --warmup 20 --no-cpu > gpurun_out/prof_online_be_$TAG.json 2> gpurun_out/prof_online_be_$TAG.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_adapter_$TAG -o run --output-format csv -- tests/cpp/build/adapter_run bench 41 3000 > gpurun_out/prof_adapter_$TAG.json 2> gpurun_out/prof_adapter_$TAG.err || exit $?
  echo "traces done"
fi
