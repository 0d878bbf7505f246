"""Per-kernel summary (and optionally a dispatch timeline) of a rocprofv3
SQLite output (run_results.db), the same figures as --stats' CSV.

  python tools/rocpd_summary.py gpurun_out/prof_x/run_results.db [--timeline N] [--grep NAME]
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"csm::\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*$", "", name)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", type=int, default=0, help="print the last N dispatches")
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, start, end, duration, grid_x, workgroup_x, lds_size, vgpr_count, "
                       "accum_vgpr_count, sgpr_count from kernels order by start").fetchall()
    rows = [r for r in rows if a.grep in r[0]]
    agg = {}
    for r in rows:
        k = short(r[0])
        n, t, mn, mx = agg.get(k, (0, 0, float("inf"), 0))
        agg[k] = (n + 1, t + r[3], min(mn, r[3]), max(mx, r[3]))
    total = sum(v[1] for v in agg.values()) or 1
    print(f"{'kernel':72s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>9s} {'%':>6s}")
    for k, (n, t, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:72s} {n:6d} {t / 1e6:10.3f} {t / n / 1e3:10.2f} {mn / 1e3:9.2f} {mx / 1e3:9.2f} "
              f"{100.0 * t / total:6.1f}")
    if a.timeline:
        t0 = rows[-a.timeline][1]
        print("\nstart_us   dur_us  gap_us  grid  wg  lds  vgpr+agpr sgpr  kernel")
        prev = None
        for r in rows[-a.timeline:]:
            gap = (r[1] - prev) / 1e3 if prev is not None else 0.0
            print(f"{(r[1] - t0) / 1e3:8.1f} {r[3] / 1e3:8.2f} {gap:7.1f} {r[4]:7d} {r[5]:4d} {r[6]:6d} "
                  f"{r[7]:4d}+{r[8]:<4d} {r[9]:4d}  {short(r[0])}")
            prev = r[2]


if __name__ == "__main__":
    main()
