#!/bin/bash
# r04 (second session): the whole GPU suite, the isolated box-kernel variants of every level
# (v11 pair default, v10 palette, v9 grouped), then the default config-2 bench line.
set -o pipefail
mkdir -p gpurun_out
T=${1:-s2}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_${T}.log 2>&1 || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -2 gpurun_out/pytest_${T}.log
out=gpurun_out/kbench_${T}.txt
: > $out
for env in "CSM_BOX_PAIR=1" "CSM_BOX_PAIR=0" "CSM_BOX_PALETTE=0"; do
  echo "# $env" >> $out
  env $env timeout -k 10 200 python tools/box_kbench.py >> $out 2>&1 || exit $?
done
for l in 1 2; do echo "# level $l" >> $out; timeout -k 10 200 python tools/box_kbench.py --level $l >> $out 2>&1 || exit $?; done
grep '^[{#]' $out
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err \
  || { tail -20 gpurun_out/bench_${T}.err; exit 1; }
python3 - gpurun_out/bench_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print(round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 4), "ms/step finish", round(d["finish_ms_per_step"], 3),
      "share", round(d["kernel_share_of_step"], 3), "host_inputs", d.get("value_host_inputs"))
for k in d["kernels"]:
    if k["name"].startswith(("score_", "finish_kernel")):
        print(" ", k["name"], k["launches"], round(k["total_ms"] / k["launches"], 4))
PY
timeout -k 10 300 python bench.py --workload online --steps 400 --warmup 20 > gpurun_out/online_${T}.json \
  2> gpurun_out/online_${T}.err || { tail -20 gpurun_out/online_${T}.err; exit 1; }
python3 - gpurun_out/online_${T}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
c = d["config"]
print("online", round(d["value"], 1), "scans/s", c["latency_ms"])
print(json.dumps(c["latency_tail"])[:3000])
PY
