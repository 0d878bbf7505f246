# Round-end measurements on one GPU (each part one gpurun call):
#   ROUND=r06 tools/gpu_round_final.sh tests     the whole GPU suite, smoke(), the tie stress
#   ROUND=r06 tools/gpu_round_final.sh pmcbench  PMC passes of this build (copied where bench.py
#                                                reads them: profiles/$ROUND), then every bench line
#                                                and the rocprofv3 kernel traces
# Results land under gpurun_out/$ROUND/.
set -o pipefail
R=${ROUND:-r06}
O=gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
case "$1" in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log
  timeout -k 10 300 python tools/stress_ties.py --iters 60 > $O/stress_ties.json 2>&1 || exit $?
  head -c 120 $O/stress_ties.json; echo ;;
pmc)
  bash tools/pmc_roofline.sh $O/pmcr || exit $?
  bash tools/pmc_roofline.sh $O/pmcb --levels sim --steps 2 --warmup 1 --no-cpu --no-latency --no-lc-leg \
    --no-host-inputs || exit $?
  bash tools/pmc_roofline.sh $O/pmclc --workload loop_closure --steps 2 --warmup 1 --no-cpu || exit $?
  bash tools/pmc_roofline.sh $O/pmcw --workload willow --steps 2 --warmup 1 --no-cpu || exit $?
  bash tools/pmc_roofline.sh $O/pmcs --workload online --steps 100 --warmup 10 --no-cpu || exit $?
  # config 4 as SURVEY 8d defines it: the whole willow map (search and exhaustive), and the tiled 15360^2 grid
  bash tools/pmc_roofline.sh $O/pmcww --workload willow --whole-map --steps 2 --warmup 1 --no-cpu || exit $?
  bash tools/pmc_roofline.sh $O/pmcwe --workload willow --whole-map --search exhaustive --steps 2 --warmup 1 --no-cpu || exit $?
  bash tools/pmc_roofline.sh $O/pmcg --workload willow --grid-cells 15360 --search exhaustive --windows 64 --steps 2 --warmup 1 --no-cpu || exit $?
  cp $O/pmcg/counters.json $O/counters_grid15k.json
  python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
a = json.load(open(f'{o}/pmcww/counters.json'))
b = json.load(open(f'{o}/pmcwe/counters.json'))
assert a['source_digest'] == b['source_digest']
for k, v in b['kernels'].items():
    a['kernels'].setdefault(k, v)
json.dump(a, open(f'{o}/counters_willow_whole.json', 'w'), indent=1)
PY
  cp $O/pmcs/counters.json $O/counters_small.json
  cp $O/pmcb/counters.json $O/counters_b109.json
  python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
a = json.load(open(f'{o}/pmclc/counters.json'))
b = json.load(open(f'{o}/pmcw/counters.json'))
assert a['source_digest'] == b['source_digest']
for k, v in b['kernels'].items():
    a['kernels'].setdefault(k, v)
json.dump(a, open(f'{o}/counters_lc.json', 'w'), indent=1)
PY
  cp $O/pmcr/counters.json $O/counters.json; echo "pmc done" ;;
bench)
  timeout -k 10 600 python bench.py > $O/bench_config2.json 2> $O/bench_config2.err || exit $?
  timeout -k 10 300 python bench.py --workload loop_closure --steps 10 --warmup 2 > $O/bench_config3_loop_closure.json 2> $O/lc.err || exit $?
  timeout -k 10 300 python bench.py --workload willow --steps 20 --warmup 3 > $O/bench_config4_willow.json 2> $O/willow.err || exit $?
  timeout -k 10 300 python bench.py --workload willow --whole-map --steps 5 --warmup 1 --cpu-seconds 8 --counters-json profiles/$R/counters_willow_whole.json > $O/bench_config4_willow_whole.json 2> $O/willow_whole.err || exit $?
  timeout -k 10 300 python bench.py --workload willow --whole-map --search exhaustive --steps 3 --warmup 1 --no-cpu --counters-json profiles/$R/counters_willow_whole.json > $O/bench_config4_willow_whole_exhaustive.json 2> $O/willow_whole_exh.err || exit $?
  timeout -k 10 400 python bench.py --workload willow --grid-cells 15360 --search exhaustive --windows 64 --steps 3 --warmup 1 --cpu-seconds 8 --counters-json profiles/$R/counters_grid15k.json > $O/bench_config4_grid15k_exhaustive.json 2> $O/grid15k.err || exit $?
  timeout -k 10 300 python bench.py --workload online --steps 400 --warmup 20 > $O/bench_config5_online.json 2> $O/online.err || exit $?
  timeout -k 10 300 python bench.py --workload online --attach-backend --rate-hz 40 --steps 300 --warmup 20 > $O/bench_config5_online_backend_40hz.json 2> $O/online_be.err || exit $?
  timeout -k 10 300 python bench.py --workload adapter --steps 40 > $O/bench_adapter.json 2> $O/adapter.err || exit $?
  timeout -k 10 300 python bench.py --workload backend > $O/bench_backend.json 2> $O/backend.err || exit $?
  rm -rf $O/prof_config2 $O/prof_b109 $O/prof_online
  # whole level-parts per dispatch (CSM_FIRST_WINDOWS=0): the summary's
  # per-dispatch averages are then the bench line's per-launch times
  CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_config2 -o run --output-format csv -- python3 bench.py --no-cpu --no-latency --no-b109 --no-lc-leg --no-host-inputs > $O/prof_config2.json 2> $O/prof_config2.err || exit $?
  CSM_FIRST_WINDOWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b109 -o run --output-format csv -- python3 bench.py --levels sim --no-cpu --no-latency --no-lc-leg --no-host-inputs > $O/prof_b109.json 2> $O/prof_b109.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_online -o run --output-format csv -- python3 bench.py --workload online --steps 200 --warmup 20 --no-cpu > $O/prof_online.json 2> $O/prof_online.err || exit $?
  echo "bench done" ;;
pmcbench)
  # one call: counters of this build, copied where bench.py reads them, then every bench line
  bash "$0" pmc || exit $?
  mkdir -p profiles/$R
  cp $O/counters.json $O/counters_b109.json $O/counters_lc.json $O/counters_small.json \
     $O/counters_willow_whole.json $O/counters_grid15k.json profiles/$R/ || exit $?
  bash "$0" bench || exit $? ;;
*) echo "usage: $0 tests|pmc|bench|pmcbench"; exit 2 ;;
esac
