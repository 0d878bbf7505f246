# A/B of the few-window path knobs (tools/small_ab.py) + the small-path tests.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_small.py tests/test_gpu_gridmap.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for cfg in ${CFGS:-"" "CSM_SPLIT_TARGET=256" "CSM_SPLIT_TARGET=1024" "CSM_SMALL=0"}; do
  env $cfg timeout -k 10 120 python tools/small_ab.py 300 > gpurun_out/small_ab_${TAG}.json 2>&1 || exit $?
  echo "[$cfg] $(cat gpurun_out/small_ab_${TAG}.json)"
done
