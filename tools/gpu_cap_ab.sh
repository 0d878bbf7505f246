# Willow and loop-closure query time against the default node capacity
# (CSM_NODE_CAPACITY), interleaved.
set -o pipefail
for rep in 1 2; do
for cap in 16777216 67108864; do
  for w in willow loop_closure; do
    CSM_NODE_CAPACITY=$cap timeout -k 10 200 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu > gpurun_out/cap.json 2> gpurun_out/cap.err || exit $?
    python3 -c "
import json;d=json.loads(open('gpurun_out/cap.json').read().strip().splitlines()[-1])
print('$w cap $cap', round(d['ms_per_step'],4), d['search'].get('same_answer_as_exhaustive'), d['search'].get('syncs_last_query'))"
  done
done
done
