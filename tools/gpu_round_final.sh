# Round-end measurements on one GPU for the current build: the GPU suite and
# smoke(), config-2 PMC passes + bench line + kernel trace, the loop-closure
# and willow PMC passes (merged into counters_lc.json) + their bench lines.
set -o pipefail
bash tools/gpu_final.sh || exit $?
bash tools/pmc_roofline.sh gpurun_out/pmclc --workload loop_closure --steps 2 --warmup 1 --no-cpu || exit $?
bash tools/pmc_roofline.sh gpurun_out/pmcw --workload willow --steps 2 --warmup 1 --no-cpu || exit $?
python3 - <<'PY'
import json
a = json.load(open('gpurun_out/pmclc/counters.json'))
b = json.load(open('gpurun_out/pmcw/counters.json'))
assert a['source_digest'] == b['source_digest']
for k, v in b['kernels'].items():
    a['kernels'].setdefault(k, v)
json.dump(a, open('gpurun_out/counters_lc_merged.json', 'w'), indent=1)
json.dump(a, open('profiles/r02/counters_lc.json', 'w'), indent=1)
PY
timeout -k 10 300 python bench.py --workload loop_closure --steps 5 --warmup 2 > gpurun_out/lc_final.json 2> gpurun_out/lc_final.err || exit $?
timeout -k 10 300 python bench.py --workload willow --steps 5 --warmup 1 > gpurun_out/willow_final.json 2> gpurun_out/willow_final.err || exit $?
echo "round final done"
