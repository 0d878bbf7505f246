"""Turn rocprofv3 --pmc CSV output into per-kernel HBM bytes per launch.

Usage: python tools/pmc_traffic.py OUT.json FETCH_DIR [WRITE_DIR]

Each DIR is a rocprofv3 -d output directory of one `--pmc` pass
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950: TCC slots,
MI355X_MICROARCH.md "rocprofv3 PMC slots"). Counters are in KiB per dispatch.
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE tallies 128-B
fabric read requests at 64 B, so the read side is doubled; WRITE_SIZE is
taken as is. Both raw and corrected figures are written.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _short(name: str) -> str:
    """rocprof's demangled name -> the name csm_kernel_stats reports."""
    key = "score_cols_kernel<"
    if key in name:  # template <int KT, bool INT, bool BEST>
        i = name.index(key) + len(key)
        kt, integer, best = [a.strip() for a in name[i:name.index(">", i)].split(",")]
        return (f"score_cols_kernel<{kt},{'int' if integer == 'true' else 'f64'},"
                f"{'best' if best == 'true' else 'all'}>")
    for key in ("score_rowsd_kernel<", "score_rows_kernel<"):  # <int NS, int SQ, bool BEST[, int BS]>
        if key in name:
            i = name.index(key) + len(key)
            ns, sq, best = [a.strip() for a in name[i:name.index(">", i)].split(",")][:3]
            return f"{key[:-1]}<{ns},{sq},{'best' if best == 'true' else 'all'}>"
    for key in ("score_box_palette_kernel<", "score_box_pair_kernel<"):  # <int NS, bool BEST[, bool NORUN]>: v10, v11
        if key in name:
            i = name.index(key) + len(key)
            args = [a.strip() for a in name[i:name.index(">", i)].split(",")]
            return f"{key[:-1]}<{args[0]},{'best' if args[1] == 'true' else 'all'}>"
    key = "score_box_grouped_kernel<"
    if key in name:  # <int NS, bool BEST>: the v9 box kernel, accounted as score_box_kernel
        i = name.index(key) + len(key)
        args = [a.strip() for a in name[i:name.index(">", i)].split(",")]
        return f"score_box_kernel<{args[0]},{'best' if args[-1] == 'true' else 'all'}>"
    key = "score_box_kernel<"
    if key in name:  # <int NS, int D, bool BEST>
        i = name.index(key) + len(key)
        args = [a.strip() for a in name[i:name.index(">", i)].split(",")]
        return f"score_box_kernel<{args[0]},{'best' if args[-1] == 'true' else 'all'}>"
    key = "pyr_topbox_kernel<"
    if key in name:  # <int NP, int NL>
        i = name.index(key) + len(key)
        args = [a.strip() for a in name[i:name.index(">", i)].split(",")]
        return f"pyr_topbox_kernel<{args[0]},{args[1]}>"
    key = "pyr_bound_kernel<"
    if key in name:  # <typename T>: the search's level passes (csm_api.cpp accounts them per depth)
        i = name.index(key) + len(key)
        return f"pyr_bound_kernel<{name[i:name.index('>', i)].strip()}>"
    key = "score_tiny_kernel<"
    if key in name:  # <int NS, bool BEST>
        i = name.index(key) + len(key)
        args = [a.strip() for a in name[i:name.index(">", i)].split(",")]
        return f"score_tiny_kernel<{args[0]},{'best' if args[-1] == 'true' else 'all'}>"
    key = "score_phase_kernel<"
    if key in name:  # <int NS, int C, int NQ, bool BEST[, bool ST]> (r04: the strip form's flag last)
        i = name.index(key) + len(key)
        args = [a.strip() for a in name[i:name.index(">", i)].split(",")]
        return f"score_phase_kernel<{args[0]},{'best' if args[3] == 'true' else 'all'}>"
    for key in ("score_all_kernel<", "score_best_kernel<"):
        if key in name:
            i = name.index(key)
            return name[i:name.index(">", i) + 1]
    for key in ("finish_fast_kernel", "finish_kernel", "analyze_grid_kernel", "fixed_point_kernel",
                "reduce_best_kernel", "score_tree_kernel", "score_split_kernel"):
        if key in name:
            return key
    return name[:64]


def read_pass(d: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            per[_short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    out, fetch_dir = sys.argv[1], sys.argv[2]
    write_dir = sys.argv[3] if len(sys.argv) > 3 else None
    fp = read_pass(fetch_dir)
    wp = read_pass(write_dir) if write_dir else {}
    res = {}
    for k, ctr in fp.items():
        f = ctr.get("FETCH_SIZE", [])
        w = wp.get(k, {}).get("WRITE_SIZE", []) if wp else []
        fkb = sum(f) / len(f) if f else 0.0
        wkb = sum(w) / len(w) if w else 0.0
        res[k] = {
            "dispatches": len(f),
            "fetch_kib_raw": fkb,
            "write_kib_raw": wkb,
            "hbm_bytes_per_launch": (2.0 * fkb + wkb) * 1024.0,
            "correction": "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B), WRITE_SIZE x1",
        }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, v in res.items():
        print(f"{k:40s} {v['dispatches']:5d} {v['hbm_bytes_per_launch'] / 1e6:12.2f} MB/launch")


if __name__ == "__main__":
    main()
