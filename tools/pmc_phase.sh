#!/bin/bash
# PMC passes (counters only, one rocprofv3 run each) over a short bench, for
# the per-kernel instruction mix and stall picture: tools/pmc_phase.sh OUT
set -e
OUT=${1:-gpurun_out/pmcp}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-latency"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d "$OUT/sq1" -- $B > "$OUT/sq1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/sq2" -- $B > "$OUT/sq2.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/ta" -- $B > "$OUT/ta.log" 2>&1
python3 tools/pmc_summary.py "$OUT/sq1" "$OUT/sq2" "$OUT/ta" > "$OUT/summary.txt"
