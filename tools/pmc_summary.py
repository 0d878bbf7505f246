"""Average rocprofv3 --pmc counters per kernel over every pass directory given."""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import _short  # noqa: E402

agg = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[_short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if "rocclr" in k or "analyze" in k or "fixed_point" in k:
        continue
    print(k)
    for c, xs in sorted(v.items()):
        print(f"   {c:32s} {sum(xs) / len(xs):16.1f}")
