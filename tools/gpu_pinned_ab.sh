# Online front end (config 5) and willow: the pinned-staging build against the
# previous library (CSM_LIB=ab_old/libroborts_csm.so), interleaved.
set -o pipefail
for rep in 1 2; do
  for lib in ab_old/libroborts_csm.so ""; do
    CSM_LIB=$lib timeout -k 10 300 python bench.py --workload online --no-cpu > gpurun_out/on.json 2> gpurun_out/on.err || exit $?
    python3 -c "
import json;d=json.loads(open('gpurun_out/on.json').read().strip().splitlines()[-1])
print('online lib=${lib:-new}', round(d['value'],1), d['unit'], round(d['ms_per_step'],4))"
  done
done
