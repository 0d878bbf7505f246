# Config-2 step time against the pool workers' spin window (CSM_POOL_SPIN_US)
# and thread count, interleaved. Usage: bash tools/gpu_pool_spin.sh
set -o pipefail
for rep in 1 2; do
for cfg in "16 0" "16 300" "16 2000" "8 0" "8 2000"; do
  set -- $cfg
  CSM_HOST_THREADS=$1 CSM_POOL_SPIN_US=$2 timeout -k 10 200 python bench.py --no-cpu --no-latency --no-b109 --steps 30 --warmup 3 > gpurun_out/ps.json 2> gpurun_out/ps.err || exit $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/ps.json').read().strip().splitlines()[-1])
h={k['name']:round(k['total_ms']/k['launches'],3) for k in d['kernels'] if k['name'].startswith('host:') and '<' in k['name']}
print('threads $1 spin $2', round(d['ms_per_step'],3), h)"
done
done
