# Exact-finish waves per window A/B (4 = the default build, 8 and 16 =
# lib/libroborts_csm-fw{8,16}.so): the parity tests under each, then
# interleaved config-2 benches with the exact pass's per-level time.
set -o pipefail
mkdir -p gpurun_out
for v in fw8 fw16; do
  CSM_LIB=$PWD/roborts-edu-slam_amd/lib/libroborts_csm-$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { echo "parity $v failed"; tail -5 gpurun_out/pytest_$v.log; exit 1; }
  echo "parity $v ok"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for v in base fw8 fw16; do
    if [ $v = base ]; then lib=""; else lib=$PWD/roborts-edu-slam_amd/lib/libroborts_csm-$v.so; fi
    rm -rf gpurun_out/prof_$v
    CSM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-latency --no-b109 > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || exit $?
    python3 - "$v" <<'PY'
import csv, json, sys, collections, glob
v = sys.argv[1]
f = glob.glob(f'gpurun_out/prof_{v}/**/*kernel_trace.csv', recursive=True)[0]
r = sorted(csv.DictReader(open(f)), key=lambda x: int(x['Start_Timestamp']))
agg = collections.defaultdict(list); cur = None
for x in r:
    n = x['Kernel_Name']; d = (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3
    for key, lv in (('score_box', 'coarse'), ('score_phase', 'fine'), ('score_tiny', 'super')):
        if key in n: cur = lv
    if 'finish_kernel' in n and 'fast' not in n: agg[cur].append(d)
d = json.loads(open(f'gpurun_out/bench_{v}.json').read().strip().splitlines()[-1])
print(v, 'ms_per_step', round(d['ms_per_step'], 3), {k: round(sum(a) / len(a), 1) for k, a in agg.items()})
PY
  done
done
