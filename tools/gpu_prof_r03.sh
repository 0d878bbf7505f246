# r03: kernel traces of the reference-configuration paths (1 cm fine map,
# integer window steps): the online front end and the drop-in adapter.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03a}
timeout -k 10 300 python bench.py --workload online --steps 200 --warmup 20 > gpurun_out/online_$TAG.json 2> gpurun_out/online_$TAG.err || exit $?
echo "online done"
timeout -k 10 300 python bench.py --workload adapter --steps 40 > gpurun_out/adapter_$TAG.json 2> gpurun_out/adapter_$TAG.err || exit $?
echo "adapter done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_online_$TAG -o run --output-format csv -- python3 bench.py --workload online --steps 200 --warmup 20 --no-cpu > gpurun_out/prof_online_$TAG.json 2> gpurun_out/prof_online_$TAG.err || exit $?
echo "online prof done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_adapter_$TAG -o run --output-format csv -- tests/cpp/build/adapter_run bench 41 3000 > gpurun_out/prof_adapter_$TAG.json 2> gpurun_out/prof_adapter_$TAG.err || exit $?
echo "adapter prof done"
