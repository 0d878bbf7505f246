# Config-2 A/B over environment knobs (each a full bench.py run, 30 steps).
# Prints scorings/s, ms per step, the kernel share of the step and the host's
# per-phase waits / work (host:* entries of the bench's kernel stats, per step).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --no-latency --no-b109 > gpurun_out/cfg2ab.json 2> gpurun_out/cfg2ab.err || exit $?
  python3 -c "
import json
d = json.load(open('gpurun_out/bench_detail.json'))  # the whole result (the last stdout line is the compact one)
print('[$cfg]', round(d['value'] / 1e9, 3), 'G', round(d['ms_per_step'], 3), 'ms share', round(d['kernel_share_of_step'], 3))
steps = d['steps']
for k in d['kernels']:
    if k['name'].startswith('host:'):
        print('   %-34s %8.3f ms/step  %6.1f calls/step' % (k['name'], k['total_ms'] / steps, k['launches'] / steps))
    elif k['name'].startswith('finish:exact_windows<'):
        print('   %-34s %6.1f of %6.1f windows per launch take the exact pass' % (k['name'],
              k['scorings'] / k['launches'], k['algorithmic_bytes'] / k['launches']))
    elif not k['name'].startswith('pool:') and k['launches']:
        print('   %-34s %8.3f ms/step  %6.1f calls/step  %7.1f us/call' % (k['name'], k['total_ms'] / steps,
              k['launches'] / steps, k['total_ms'] / k['launches'] * 1e3))
    elif k['name'].startswith('pool:'):
        print('   %-34s first worker joins %6.1f us after the notify, caller ran %4.0f %% of the items'
              % (k['name'], k['total_ms'] / k['launches'] * 1e3, 100 * k['algorithmic_bytes'] / k['launches']))
"
done
