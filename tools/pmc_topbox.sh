# Counter passes over the loop-closure bench (the pyramid top kernel), one
# rocprofv3 --pmc run per pass, merged by tools/pmc_roofline.py.
set -e
OUT=gpurun_out/pmc_lc
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--workload loop_closure --steps 2 --warmup 1 --no-cpu"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -- python3 bench.py $ARGS \
    > "$OUT/$name.json" 2> "$OUT/$name.err"
  echo "pass $name done"
}
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE
run sq2 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
python3 tools/pmc_roofline.py "$OUT/counters.json" "$OUT"/tcc "$OUT"/sq1 "$OUT"/sq2 "$OUT"/fetch > "$OUT/summary.txt"
