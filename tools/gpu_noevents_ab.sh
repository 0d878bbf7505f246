cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --no-latency --no-b109 > gpurun_out/ne.json 2> gpurun_out/ne.err || exit $?
  python3 -c "
import json
d = json.loads(open('gpurun_out/ne.json').read().strip().splitlines()[-1])
print('[$cfg]', round(27.0e6 * 1e3 / d['ms_per_step'] / 1e9, 3), 'G (27.0 M scorings per step)', round(d['ms_per_step'], 3), 'ms')
"
done
