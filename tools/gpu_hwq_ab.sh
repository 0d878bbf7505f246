# The exact finish pass on its own stream (CSM_EXACT_STREAM=1) or not, with 4
# (default) or 8 hardware queues per process: config-2 step, 30 steps per run.
set -o pipefail
for i in 1 2 3; do
  for cfg in "4 0" "4 1" "8 0" "8 1"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 CSM_EXACT_STREAM=$2 timeout -k 10 200 python bench.py --no-cpu --no-latency --no-b109 --steps 30 --warmup 3 > gpurun_out/hwq.json 2> gpurun_out/hwq.err || exit $?
    python3 -c "
import json; d = json.loads(open('gpurun_out/hwq.json').read().strip().splitlines()[-1])
print('hwq=$1 xstream=$2 run $i', round(d['ms_per_step'], 3))"
  done
done
