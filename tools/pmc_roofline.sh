#!/bin/bash
# PMC passes for bench.py's roofline (run on the GPU box from the repo root):
#   tools/pmc_roofline.sh OUT [bench args...]
# One rocprofv3 run per pass, counters only (no trace domains), each pass within
# the per-block limits (<= 8 SQ, 4 TCC, 2 TA, 2 GRBM). Then
# tools/pmc_roofline.py merges them into OUT/counters.json.
set -e
OUT=${1:-gpurun_out/pmcr}
shift || true
ARGS=${*:-"--steps 2 --warmup 1 --no-cpu --no-latency --no-b109 --no-lc-leg"}
mkdir -p "$OUT"
export TMPDIR=/tmp
# every scoring dispatch a whole level-part (the 3-level driver otherwise
# scores its first part's coarse level in two spans): counters per dispatch
# then match bench.py's per-launch HIP-event times
export CSM_FIRST_WINDOWS=0
run() {  # run NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -- python3 bench.py $ARGS \
    > "$OUT/$name.json" 2> "$OUT/$name.err"
}
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
run write WRITE_SIZE GRBM_GUI_ACTIVE
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE
run sq2 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE
F64=""
for c in SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64; do
  if grep -qw "$c" "$OUT/counters_list.txt"; then F64="$F64 $c"; fi
done
if [ -n "$F64" ]; then run f64 $F64 GRBM_GUI_ACTIVE; fi
python3 tools/pmc_roofline.py "$OUT/counters.json" "$OUT"/fetch "$OUT"/write "$OUT"/sq1 "$OUT"/sq2 \
  $( [ -n "$F64" ] && echo "$OUT/f64" ) > "$OUT/summary.txt"
