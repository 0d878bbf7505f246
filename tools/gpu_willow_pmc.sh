# PMC passes over the willow leg (its top-level kernel instantiation), merged
# into profiles/r02/counters_lc.json beside the loop-closure leg's kernels,
# then the willow leg with its roofline.
set -o pipefail
bash tools/pmc_roofline.sh gpurun_out/pmcw --workload willow --steps 2 --warmup 1 --no-cpu || exit $?
python3 - <<'PY'
import json
a = json.load(open('profiles/r02/counters_lc.json'))
b = json.load(open('gpurun_out/pmcw/counters.json'))
assert a['source_digest'] == b['source_digest']
for k, v in b['kernels'].items():
    a['kernels'].setdefault(k, v)
json.dump(a, open('profiles/r02/counters_lc.json', 'w'), indent=1)
json.dump(a, open('gpurun_out/counters_lc_merged.json', 'w'), indent=1)
PY
timeout -k 10 300 python bench.py --workload willow --steps 5 --warmup 1 > gpurun_out/willow_final.json 2> gpurun_out/willow_final.err || exit $?
echo done
