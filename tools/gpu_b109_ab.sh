# B = 109 leg A/B: default build (tiny-window super-fine kernel) vs
# CSM_KERNEL=v7 (the LDS-DMA row kernel for the super-fine level), interleaved.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for m in default v7; do
    if [ $m = default ]; then e=""; else e="CSM_KERNEL=v7"; fi
    env $e timeout -k 10 200 python bench.py --no-cpu --no-latency > gpurun_out/b109_${m}_$i.json 2> gpurun_out/b109_${m}_$i.err || exit $?
    python3 -c "
import json; d = json.loads(open('gpurun_out/b109_${m}_$i.json').read().strip().splitlines()[-1])
ks = {k['name']: round(k['total_ms'] / k['launches'], 3) for k in d['b109'].get('kernels', [])} if isinstance(d.get('b109'), dict) else {}
print('$m', $i, round(d['ms_per_step'], 3), round(d['b109']['ms_per_step'], 3), ks)"
  done
done
