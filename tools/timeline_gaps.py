"""Idle time of the kernel stream in config-2 steps, from a rocprofv3
--kernel-trace CSV (tools/gpu_r03_final.sh trace2, or any bench run under
rocprofv3): the gaps between consecutive kernels of the queue the scoring
kernels run on, summed by (kernel before, kernel after), per step.

  python tools/timeline_gaps.py gpurun_out/prof/.../run_kernel_trace.csv [steps] [parts]
"""
import collections
import csv
import sys


def short(name):
    for k in ("score_box_pair_kernel", "score_box_grouped_kernel", "score_box_kernel", "score_phase_kernel", "score_tiny_kernel",
              "finish_fast_kernel", "finish_kernel", "fillBuffer", "copyBuffer"):
        if k in name:
            return k
    return name[:28]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    by_q = collections.defaultdict(list)
    for r in rows:
        by_q[r[qkey]].append(r)
    # the scoring queue: the one holding the phase kernels
    main_q = max(by_q, key=lambda q: sum("score_phase" in r["Kernel_Name"] for r in by_q[q]))
    seq = by_q[main_q]
    # a step starts at a coarse (box) launch that follows a tiny-window launch's finish
    starts = [i for i, r in enumerate(seq) if "score_box" in r["Kernel_Name"] and i > 0 and
              any("score_tiny" in seq[j]["Kernel_Name"] for j in range(max(0, i - 3), i))]
    starts = starts[-(steps + 1):]
    if len(starts) < 2:
        sys.exit("fewer than two steps found")
    gaps = collections.Counter()
    busy = collections.Counter()
    n = 0
    t_total = 0.0
    # steps: tiny-window launches / parts (a step's coarse launches can come
    # in two spans and the parts interleave across batches)
    parts = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    a, b = starts[0], starts[-1]
    n = max(1, sum("score_tiny" in seq[i]["Kernel_Name"] for i in range(a, b)) // parts)
    t_total = (int(seq[b]["Start_Timestamp"]) - int(seq[a]["Start_Timestamp"])) / 1e3
    if True:
        for i in range(a, b):
            r, nx = seq[i], seq[i + 1]
            busy[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            g = (int(nx["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3
            gaps[(short(r["Kernel_Name"]), short(nx["Kernel_Name"]))] += max(g, 0.0)
    print(f"{n} steps, {t_total / n:.1f} us per step on queue {main_q}")
    print("busy per step:")
    for k, v in busy.most_common():
        print(f"   {k:28s} {v / n:8.1f} us")
    print(f"   {'(sum)':28s} {sum(busy.values()) / n:8.1f} us")
    print("idle per step, by transition:")
    for (p, q), v in gaps.most_common():
        print(f"   {p:26s} -> {q:26s} {v / n:8.1f} us")
    print(f"   {'(sum)':55s} {sum(gaps.values()) / n:8.1f} us")
    others = [q for q in by_q if q != main_q]
    t0, t1 = int(seq[starts[0]]["Start_Timestamp"]), int(seq[starts[-1]]["Start_Timestamp"])
    for q in others:
        rs = [r for r in by_q[q] if t0 <= int(r["Start_Timestamp"]) < t1]
        if rs:
            tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e3
            names = collections.Counter(short(r["Kernel_Name"]) for r in rs)
            print(f"queue {q}: {len(rs) / n:.1f} kernels, {tot / n:.1f} us per step ({dict(names)})")


if __name__ == "__main__":
    main()
