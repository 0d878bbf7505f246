#!/bin/bash
# PMC passes for the bench workload (run on the GPU box from the repo root).
# Each pass is its own rocprofv3 run with counters only (no trace domains).
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-latency"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -- $B > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -- $B > "$OUT/write.json" 2> "$OUT/write.err"
python3 tools/pmc_traffic.py "$OUT/traffic.json" "$OUT/fetch" "$OUT/write" > "$OUT/traffic.txt"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -k 10 240 rocprofv3 --pmc ${PMC_SQ:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES} --output-format csv -d "$OUT/sq" -- $B > "$OUT/sq.json" 2> "$OUT/sq.err"
timeout -k 10 240 rocprofv3 --pmc ${PMC_T:-TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum} --output-format csv -d "$OUT/ta" -- $B > "$OUT/ta.json" 2> "$OUT/ta.err"
