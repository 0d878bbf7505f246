# Config-2 step time and per-level host plan/complete times (ms per call)
# against CSM_HOST_THREADS. Usage: bash tools/gpu_host_threads.sh "1 16"
set -o pipefail
for t in ${1:-1 2 4 8 16}; do
  CSM_HOST_THREADS=$t timeout -k 10 200 python bench.py --no-cpu --no-latency --no-b109 --steps 20 --warmup 3 > gpurun_out/ht.json 2> gpurun_out/ht.err || exit $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/ht.json').read().strip().splitlines()[-1])
h={k['name']:round(k['total_ms']/k['launches'],3) for k in d['kernels'] if k['name'].startswith('host:') and '<' in k['name']}
print('threads $t', round(d['ms_per_step'],3), h)"
done
