#!/bin/bash
# r04: which HIP calls make scan 42 of the config-5 stream slow (tools/online_probe.py under a HIP API trace)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/probe42
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/probe42 -o run --output-format csv -- \
  python3 tools/online_probe.py 42 > gpurun_out/probe42.txt 2> gpurun_out/probe42.err || { tail -20 gpurun_out/probe42.err; exit 1; }
f=$(find gpurun_out/probe42 -name '*hip_api_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
longest = sorted(rows, key=dur, reverse=True)[:25]
t0 = min(int(r["Start_Timestamp"]) for r in rows)
for r in longest:
    print("%10.1f us  at %12.1f ms  %s" % (dur(r), (int(r["Start_Timestamp"]) - t0) / 1e6, r["Function"]))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    a = agg[r["Function"]]; a[0] += 1; a[1] += dur(r)
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
    print("%-40s %7d calls %10.1f us" % (k, n, t))
PY
cut -c1-300 gpurun_out/probe42.txt
