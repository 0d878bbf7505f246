# A/B of the default library against a variant build (make VARIANT=NAME ...),
# headline and B = 109, interleaved, after the driver's parity tests on the
# default build:  tools/gpu_ab_lib.sh NAME [ROUNDS]
set -o pipefail
mkdir -p gpurun_out
V=$1; R=${2:-3}
L=roborts-edu-slam_amd/lib/libroborts_csm-$V.so
[ -f "$L" ] || { echo "no $L"; exit 2; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "pipelined or submitted or timed or host_signal or staged or drop_queued" > gpurun_out/pytest_ab_$V.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ab_$V.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=$R bash tools/ab_bench.sh gpurun_out/ab_${V}_h.txt "X=0" "CSM_LIB=$L" || exit $?
ROUNDS=$R BENCH_ARGS="--levels sim" bash tools/ab_bench.sh gpurun_out/ab_${V}_s.txt "X=0" "CSM_LIB=$L" || exit $?
echo done
