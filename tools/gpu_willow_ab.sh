# Config-4 (willow) A/B over environment knobs: ms per query of the admissible
# search and the top kernel's live time. tools/gpu_willow_ab.sh "K=V ..." ...
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --workload willow --steps 20 --warmup 3 --no-cpu > gpurun_out/wab.json 2> gpurun_out/wab.err || exit $?
  python3 -c "
import json
d = json.loads(open('gpurun_out/wab.json').read().strip().splitlines()[-1])
k = {s['name']: s for s in d['kernels']}
top = [s for n, s in k.items() if n.startswith('pyr_topbox_kernel')]
print('[$cfg] %.3f ms/query' % d['ms_per_step'], ' top %.1f us' % (top[0]['total_ms'] / top[0]['launches'] * 1e3) if top else '',
      ' same_as_exhaustive', d['search'].get('same_answer_as_exhaustive'))
"
done
