# Round-end check on one GPU: the whole GPU suite, smoke(), the PMC passes for
# bench.py's roofline (counters for this build), then the default bench line
# and a kernel-trace summary of it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_final.log
bash tools/pmc_roofline.sh gpurun_out/pmcr || exit $?
cp gpurun_out/pmcr/counters.json profiles/r02/counters.json
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --no-cpu --no-latency > gpurun_out/prof_final.json 2> gpurun_out/prof_final.err || exit $?
echo "final done"
