"""Per-kernel dispatch-duration distribution from a rocprofv3 --kernel-trace CSV:
launches, mean, p50, p99 and max in microseconds, plus the queue each ran on.
The rocprof stats file gives only mean/min/max; the exact finish pass's tail
(a 862 us maximum against an 89 us mean) needs the distribution,
and the start of the slowest dispatches relative to the kernels beside them.

  python tools/dispatch_stats.py run_kernel_trace.csv [name-substring ...]
"""
import collections
import csv
import json
import sys


def short(name):
    name = name.split("(")[0]
    return name.replace("void ", "").replace("csm::(anonymous namespace)::", "").replace("csm::", "")[:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    pats = sys.argv[2:]
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    by_k = collections.defaultdict(list)
    for r in rows:
        k = short(r["Kernel_Name"])
        if pats and not any(p in k for p in pats):
            continue
        by_k[k].append(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r[qkey]))
    out = {}
    for k, v in sorted(by_k.items(), key=lambda kv: -sum(d for d, _ in kv[1])):
        d = sorted(x for x, _ in v)
        n = len(d)
        out[k] = {"launches": n, "mean_us": sum(d) / n, "p50_us": d[n // 2], "p99_us": d[min(n - 1, int(0.99 * n))],
                  "max_us": d[-1], "queues": sorted(set(q for _, q in v))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
