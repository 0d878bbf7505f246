# Tiny-window kernel: the parity tests, then a kernel-trace summary of the
# config-2 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tiny.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_tiny.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_tiny
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tiny -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-latency --no-b109 > gpurun_out/prof_tiny.json 2> gpurun_out/prof_tiny.err || exit $?
python3 - <<'PY'
import csv, json
for row in csv.DictReader(open('gpurun_out/prof_tiny/run_kernel_stats.csv')):
    if 'score_' in row['Name'] or 'finish' in row['Name']:
        print(f"{row['Name'][:48]:48s} {row['Calls']:>4} {float(row['AverageNs'])/1e3:9.1f} us")
d = json.loads(open('gpurun_out/prof_tiny.json').read().strip().splitlines()[-1])
print('ms_per_step', round(d['ms_per_step'], 3))
PY
