"""Isolated timing of one level's scoring kernel: config 2's 4096 scans matched
at the coarse level only (or --level 1/2; csm_scan_match_batch), unpipelined (CSM_PIPELINE=0,
CSM_FIRST_WINDOWS=0), so no other kernel of the batch runs beside it and the
HIP-event time of each launch is the kernel's own.

  python tools/box_kbench.py [--level 0] [--iters 20] [--scans 4096]

CSM_LIB selects a variant library (timing-only diagnostic builds included).
Prints one JSON line: the kernel name, launches and mean/min ms per launch.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd")]
os.environ.setdefault("CSM_PIPELINE", "0")
os.environ.setdefault("CSM_FIRST_WINDOWS", "0")

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--level", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scans", type=int, default=4096)
    a = ap.parse_args()
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.params import headline_levels
    w = worlds.make_world(2000, 2000, 0.05)
    b = worlds.make_scan_batch(w, a.scans, seed=7)
    lv = headline_levels()[a.level]
    c = roborts_csm.Context(0)
    c.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 1))
    eye = np.tile(np.eye(3).reshape(1, 9), (b.init_poses.shape[0], 1))
    for i in range(a.warmup + a.iters):
        if i == a.warmup:
            c.set_profiling(True)
        poses = np.ascontiguousarray(b.init_poses.copy())
        c.scan_match_batch(b.points_cells, b.offsets, lv, poses, eye.copy())
    st = [k for k in c.kernel_stats() if k["name"].startswith("score_")]
    out = []
    for k in st:
        out.append({"kernel": k["name"], "launches": k["launches"], "ms_per_launch": k["total_ms"] / max(1, k["launches"])})
    print(json.dumps({"level": a.level, "scans": a.scans, "lib": os.environ.get("CSM_LIB", ""), "kernels": out}),
          flush=True)
    c.close()


if __name__ == "__main__":
    main()
