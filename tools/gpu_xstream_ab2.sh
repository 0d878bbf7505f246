# Exact-pass stream A/B with longer runs (30 steps), alternating.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for m in 1 0; do
    CSM_EXACT_STREAM=$m timeout -k 10 200 python bench.py --no-cpu --no-latency --no-b109 --steps 30 --warmup 3 > gpurun_out/xs2_${m}_$i.json 2> gpurun_out/xs2_${m}_$i.err || exit $?
    python3 -c "
import json; d = json.loads(open('gpurun_out/xs2_${m}_$i.json').read().strip().splitlines()[-1])
print('exact_stream=$m run $i', round(d['ms_per_step'], 3))"
  done
done
