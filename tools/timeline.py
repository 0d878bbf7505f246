"""Kernel timeline of the last bench steps from a rocprofv3 --kernel-trace CSV:
start, duration and the idle gap before each kernel (microseconds)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 36


def short(name):
    for k in ("score_box_kernel", "score_rowsd_kernel<11", "score_rowsd_kernel<3", "finish_fast_kernel",
              "finish_kernel", "analyze", "fixed"):
        if k in name:
            return k
    return name[:24]


seq = rows[-n:]
t0 = int(seq[0]["Start_Timestamp"])
prev = None
busy = gaps = 0.0
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    busy += (e - s) / 1e3
    gaps += max(gap, 0.0)
    print(f"{short(r['Kernel_Name']):26s} start {(s - t0) / 1e3:9.1f} dur {(e - s) / 1e3:8.1f} gap {gap:8.1f}")
    prev = e
print(f"busy {busy:.1f} us, gaps {gaps:.1f} us")
