#!/bin/bash
# A/B of env settings on the default bench, interleaved (run on the GPU box
# from the repo root): tools/ab_bench.sh OUT "ENV_A" "ENV_B" ... ; each
# setting runs ROUNDS times (default 3), one ms_per_step line per run.
# BENCH_ARGS: extra bench.py arguments (e.g. "--levels sim" for B = 109).
OUT=$1; shift
ROUNDS=${ROUNDS:-3}
: > "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 120 python bench.py --no-cpu --no-latency --no-b109 --no-lc-leg --no-host-inputs --steps ${STEPS:-20} ${BENCH_ARGS:-} --detail-json gpurun_out/ab_detail.json > /dev/null 2>&1 || exit 1
    line=$(cat gpurun_out/ab_detail.json)
    ms=$(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); print("%.3f" % d["ms_per_step"], " ".join("%s=%.3f" % (k["name"].split("<")[0].replace("score_", "").replace("_kernel", "") + "<" + k["name"].split("<")[1].split(",")[0], k["total_ms"] / k["launches"]) for k in d.get("kernels", []) if k["name"].startswith(("score_", "finish_kernel")) and k["launches"]))' "$line")
    echo "$cfg $ms" | tee -a "$OUT"
  done
done
