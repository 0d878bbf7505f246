# Kernel-trace summaries of the headline (config 2) bench and of the
# loop-closure bench (config 3, pyramid search) for profiles/r02.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --workload loop_closure --steps 5 --warmup 2 --no-cpu > gpurun_out/lc_r02e.json 2> gpurun_out/lc_r02e.err || exit $?
echo "lc done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-latency --no-b109 > gpurun_out/prof_cfg2.json 2> gpurun_out/prof_cfg2.err || exit $?
echo "cfg2 prof done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lc -o run --output-format csv -- python3 bench.py --workload loop_closure --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_lc.json 2> gpurun_out/prof_lc.err || exit $?
echo "lc prof done"
