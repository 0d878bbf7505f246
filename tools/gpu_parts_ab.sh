# Config-2 step time against the pipeline part count (CSM_PIPELINE_PARTS), interleaved.
set -o pipefail
for rep in 1 2 3; do
for p in 2 3 4; do
  CSM_PIPELINE_PARTS=$p timeout -k 10 200 python bench.py --no-cpu --no-latency --no-b109 --steps 30 --warmup 3 > gpurun_out/pa.json 2> gpurun_out/pa.err || exit $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/pa.json').read().strip().splitlines()[-1])
print('parts $p', round(d['ms_per_step'],3))"
done
done
