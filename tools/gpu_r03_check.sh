# r03: GPU suite subset + online/adapter numbers for the current build.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
TESTS=${2:-tests/test_gpu_small.py}
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu $TESTS > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python bench.py --workload online --steps 200 --warmup 20 --no-cpu > gpurun_out/online_$TAG.json 2> gpurun_out/online_$TAG.err || exit $?
timeout -k 10 300 python bench.py --workload adapter --steps 40 > gpurun_out/adapter_$TAG.json 2> gpurun_out/adapter_$TAG.err || exit $?
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
for f in (f"gpurun_out/online_{t}.json", f"gpurun_out/adapter_{t}.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    c = d["config"]
    print(f, round(d["value"], 1), d["unit"], "ms/step", round(d["ms_per_step"], 4), json.dumps(c.get("latency_ms", c.get("incremental_ms_p50"))))
PY
