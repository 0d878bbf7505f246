# Copy the results of tools/gpu_round_final.sh (gpurun_out/) into profiles/r02.
set -e
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/prof_final/run_kernel_stats.csv')))
out = ["# rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --no-latency (config 2, r02 final build)",
       "# NOTE: the run includes the bench's B = 109 leg (b109), so each kernel's calls are half B = 1081 and half B = 109; the B = 1081 box average is the bench line's roofline.avg_launch_ms",
       f"{'kernel':80s} {'calls':>6s} {'avg_us':>10s} {'total_ms':>10s}"]
for r in rows[:20]:
    out.append(f"{r['Name'][:80]:80s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.1f} {float(r['TotalDurationNs'])/1e6:10.3f}")
open('profiles/r02/rocprof_kernel_stats_config2_final.txt', 'w').write("\n".join(out) + "\n")
PY
cp gpurun_out/pmcr/counters.json profiles/r02/counters.json
cp gpurun_out/pmcr/summary.txt profiles/r02/pmc_summary_config2.txt
cp gpurun_out/pmclc/summary.txt profiles/r02/pmc_summary_lc_final.txt
cp gpurun_out/pmcw/summary.txt profiles/r02/pmc_summary_willow_final.txt
cp gpurun_out/counters_lc_merged.json profiles/r02/counters_lc.json
cp gpurun_out/pytest_final.log profiles/r02/pytest_gpu_r02_final.log
tail -1 gpurun_out/bench_final.json > profiles/r02/bench_config2_r02_final.json
tail -1 gpurun_out/lc_final.json > profiles/r02/bench_config3_loop_closure_r02_final.json
tail -1 gpurun_out/willow_final.json > profiles/r02/bench_config4_willow_r02_final.json
python3 - <<'PY'
import json, sys
sys.path.insert(0, '.')
import bench
for f in ['bench_config2_r02_final', 'bench_config3_loop_closure_r02_final', 'bench_config4_willow_r02_final']:
    d = json.load(open('profiles/r02/' + f + '.json'))
    print(f, round(d['value'] / 1e9, 3), 'G', d['unit'], round(d['ms_per_step'], 3), d['roofline']['kernel'],
          round(d['roofline']['frac'], 3), d['roofline'].get('counters_stale'), (d.get('search') or {}).get('exhaustive_ms_per_query'))
print(bench.source_digest(), json.load(open('profiles/r02/counters.json'))['source_digest'],
      json.load(open('profiles/r02/counters_lc.json'))['source_digest'])
PY
