set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --levels sim --no-cpu --no-lc-leg --no-host-inputs > gpurun_out/b109_main.json 2> gpurun_out/b109_main.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_b109
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b109 -o run --output-format csv -- python3 bench.py --levels sim --no-cpu --no-latency --no-lc-leg --no-host-inputs --steps 20 --warmup 10 > gpurun_out/prof_b109.json 2> gpurun_out/prof_b109.err || exit $?
echo done
