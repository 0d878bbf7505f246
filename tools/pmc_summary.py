"""Average rocprofv3 --pmc counters per kernel over every pass directory given."""
import csv, glob, sys
from collections import defaultdict
agg = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            for key in ("score_rows_kernel<", "score_cols_kernel<", "finish_kernel"):
                if key in n:
                    i = n.index(key)
                    n = n[i:n.find(">", i) + 1] if key.endswith("<") else key
                    break
            agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if "rocclr" in k or "analyze" in k or "fixed_point" in k:
        continue
    print(k)
    for c, xs in sorted(v.items()):
        print(f"   {c:32s} {sum(xs) / len(xs):16.1f}")
