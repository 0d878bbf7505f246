# Round-4 end measurements on one GPU, in three parts (each one gpurun call):
#   tools/gpu_r04_final.sh tests   the whole GPU suite and smoke()
#   tools/gpu_r04_final.sh pmc     PMC passes: config 2 (counters.json), loop closure + willow (counters_lc.json)
#   tools/gpu_r04_final.sh bench   bench lines of every workload + rocprofv3 kernel traces
# Results land under gpurun_out/r04/; copy the pmc part's counters*.json into
# profiles/r04 before the bench part (bench.py reads them from there).
set -o pipefail
mkdir -p gpurun_out/r04
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04
case "$1" in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log ;;
pmc)
  bash tools/pmc_roofline.sh $O/pmcr || exit $?
  bash tools/pmc_roofline.sh $O/pmclc --workload loop_closure --steps 2 --warmup 1 --no-cpu || exit $?
  bash tools/pmc_roofline.sh $O/pmcw --workload willow --steps 2 --warmup 1 --no-cpu || exit $?
  bash tools/pmc_roofline.sh $O/pmcs --workload online --steps 100 --warmup 10 --no-cpu || exit $?
  cp $O/pmcs/counters.json $O/counters_small.json
  python3 - <<'PY'
import json
a = json.load(open('gpurun_out/r04/pmclc/counters.json'))
b = json.load(open('gpurun_out/r04/pmcw/counters.json'))
assert a['source_digest'] == b['source_digest']
for k, v in b['kernels'].items():
    a['kernels'].setdefault(k, v)
json.dump(a, open('gpurun_out/r04/counters_lc.json', 'w'), indent=1)
PY
  cp $O/pmcr/counters.json $O/counters.json; echo "pmc done" ;;
pmcbench)
  # one call: counters of this build, copied where bench.py reads them, then every bench line
  bash "$0" pmc || exit $?
  cp $O/counters.json $O/counters_lc.json $O/counters_small.json profiles/r04/ || exit $?
  bash "$0" bench || exit $? ;;
trace2)
  rm -rf $O/prof_config2
  CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_config2 -o run --output-format csv -- python3 bench.py --no-cpu --no-latency --no-b109 > $O/prof_config2.json 2> $O/prof_config2.err || exit $?
  echo "trace done" ;;
bench)
  # the counters of the pmc part, copied into profiles/r04 (gpurun_out does not
  # travel to the next box), feed the rooflines: bench.py's defaults
  timeout -k 10 600 python bench.py > $O/bench_config2.json 2> $O/bench_config2.err || exit $?
  timeout -k 10 300 python bench.py --workload loop_closure --steps 10 --warmup 2 > $O/bench_config3_loop_closure.json 2> $O/lc.err || exit $?
  timeout -k 10 300 python bench.py --workload willow --steps 20 --warmup 3 > $O/bench_config4_willow.json 2> $O/willow.err || exit $?
  timeout -k 10 300 python bench.py --workload online --steps 400 --warmup 20 > $O/bench_config5_online.json 2> $O/online.err || exit $?
  timeout -k 10 300 python bench.py --workload online --attach-backend --rate-hz 40 --steps 300 --warmup 20 > $O/bench_config5_online_backend_40hz.json 2> $O/online_be.err || exit $?
  timeout -k 10 300 python bench.py --workload adapter --steps 40 > $O/bench_adapter.json 2> $O/adapter.err || exit $?
  timeout -k 10 300 python bench.py --workload backend > $O/bench_backend.json 2> $O/backend.err || exit $?
  timeout -k 10 300 python bench.py --workload online --attach-backend --steps 300 --warmup 20 --no-cpu > $O/bench_config5_online_backend_unpaced.json 2> $O/online_beu.err || exit $?
  rm -rf $O/prof_config2
  # whole level-parts per dispatch (CSM_FIRST_WINDOWS=0), B = 1081 only: the
  # summary's per-dispatch averages are then the bench line's per-launch times
  CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_config2 -o run --output-format csv -- python3 bench.py --no-cpu --no-latency --no-b109 > $O/prof_config2.json 2> $O/prof_config2.err || exit $?
  rm -rf $O/prof_online $O/prof_adapter
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_online -o run --output-format csv -- python3 bench.py --workload online --steps 200 --warmup 20 --no-cpu > $O/prof_online.json 2> $O/prof_online.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_adapter -o run --output-format csv -- tests/cpp/build/adapter_run bench 41 3000 > $O/prof_adapter.json 2> $O/prof_adapter.err || exit $?
  timeout -k 10 200 python tools/online_probe.py 42 120 > $O/online_probe.txt 2> $O/online_probe.err || exit $?
  echo "bench done" ;;
*) echo "usage: $0 tests|pmc|bench"; exit 2 ;;
esac
