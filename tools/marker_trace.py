"""What the event recorded before each scoring launch changes,
from a rocprofv3 --kernel-trace --hip-trace --memory-copy-trace run of
bench.py: per scoring dispatch, (a) how long its hipLaunchKernel /
hipModuleLaunchKernel call took on the host, (b) launch call end -> kernel
start, (c) the inputs' H2D copy end -> kernel start, (d) the previous kernel's
end on the same queue -> kernel start; medians per scoring kernel.

  python tools/marker_trace.py DIR [DIR...]   (each DIR: a rocprofv3 -d output)
"""
import collections
import csv
import glob
import os
import statistics
import sys


def load(d, what):
    f = glob.glob(os.path.join(d, "**", f"*{what}.csv"), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    for d in sys.argv[1:]:
        kern = load(d, "kernel_trace")
        api = load(d, "hip_api_trace")
        cps = load(d, "memory_copy_trace")
        by_corr = {r["Correlation_Id"]: r for r in api}
        kern.sort(key=lambda r: int(r["Start_Timestamp"]))
        h2d = sorted(int(r["End_Timestamp"]) for r in cps if "HOST_TO_DEVICE" in r.get("Direction", r.get("Kind", "")))
        prev_end = {}
        stats = collections.defaultdict(lambda: collections.defaultdict(list))
        calls = collections.Counter(r["Function"] for r in api)
        for r in kern:
            q = r["Queue_Id"]
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            name = r["Kernel_Name"]
            if "score_" in name:
                k = name.split("(")[0].split("::")[-1][:40]
                a = by_corr.get(r["Correlation_Id"])
                if a is not None:
                    stats[k]["launch_call_us"].append((int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3)
                    stats[k]["call_end_to_start_us"].append((s - int(a["End_Timestamp"])) / 1e3)
                import bisect
                i = bisect.bisect_left(h2d, s) - 1
                if i >= 0:
                    stats[k]["copy_end_to_start_us"].append((s - h2d[i]) / 1e3)
                if q in prev_end:
                    stats[k]["prev_kernel_end_to_start_us"].append((s - prev_end[q]) / 1e3)
            prev_end[q] = e
        print(f"== {d}")
        for k, v in sorted(stats.items()):
            print("  " + k)
            for m, xs in v.items():
                print(f"    {m:30s} median {statistics.median(xs):9.1f}  p90 {sorted(xs)[int(0.9 * (len(xs) - 1))]:9.1f}  n {len(xs)}")
        top = ", ".join(f"{f} {n}" for f, n in calls.most_common(12))
        print(f"  HIP calls: {top}")


if __name__ == "__main__":
    main()
