# A/B of the line-shifted grid copy for the box kernel (CSM_BOX_SHIFT=1):
# parity tests under it, then interleaved config-2 benches.
set -o pipefail
mkdir -p gpurun_out
CSM_BOX_SHIFT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_shift.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_shift.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for m in 0 1; do
    CSM_BOX_SHIFT=$m timeout -k 10 200 python bench.py --no-cpu --no-b109 --no-latency > gpurun_out/bench_shift${m}_$i.json 2> gpurun_out/bench_shift${m}_$i.err || exit $?
  done
done
python3 - <<'PY'
import json
for m in (0, 1):
    for i in (1, 2, 3):
        d = json.loads(open(f'gpurun_out/bench_shift{m}_{i}.json').read().strip().splitlines()[-1])
        box = [k for k in d['kernels'] if k['name'].startswith('score_box')][0]
        print(m, i, round(d['ms_per_step'], 3), 'box avg ms', round(box['total_ms'] / box['launches'], 4))
PY
