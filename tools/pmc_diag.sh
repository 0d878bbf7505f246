#!/bin/bash
# Diagnostic counter passes for the scoring kernels (run on the GPU box).
set -e
OUT=${1:-gpurun_out/diag}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 1 --no-cpu --no-latency --scans 2048"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d "$OUT/p1" -- $B > "$OUT/p1.json" 2> "$OUT/p1.err"
timeout -k 10 240 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum --output-format csv -d "$OUT/p2" -- $B > "$OUT/p2.json" 2> "$OUT/p2.err"
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/p3" -- $B > "$OUT/p3.json" 2> "$OUT/p3.err" || true
timeout -k 10 240 rocprofv3 --pmc TD_BUSY_avr TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/p4" -- $B > "$OUT/p4.json" 2> "$OUT/p4.err" || true
