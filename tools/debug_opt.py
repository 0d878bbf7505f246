"""Localise a device/oracle divergence of the Gauss-Newton matcher: rerun one
scan with iterate_max_times = 1..T and report the first count that differs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import pyoracle as O  # noqa: E402
import roborts_csm  # noqa: E402
from roborts_csm import worlds  # noqa: E402
from roborts_csm.params import OptimizeScanMatchParam  # noqa: E402

w = worlds.make_world(2000, 2000, 0.05, seed=11)
b = worlds.make_scan_batch(w, 64, seed=12)
init = b.init_poses.copy()
init[5, :2] = [-w.offset[0] + 0.3, -w.offset[1] + 0.3]
init[9, 2] += 1.5
ctx = roborts_csm.Context(0)
ctx.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 0), force=True)
m = O.Map(w.grid, w.resolution, w.offset)
bad = []
for k in range(64):
    pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
    for t in range(1, 26):
        prm = OptimizeScanMatchParam(t, 0.0, 0.0, 0.05, 0.05)
        pose = np.array(init[k])
        c = ctx.optimize_scan_match(pts, prm, pose)
        c2, p2, it = O.optimize_scan_match(m, pts, prm, init[k])
        if c != c2 or not np.array_equal(pose, p2):
            est = O.world_to_map(m, pose)
            print(f"scan {k} diverges at iterate_max_times={t}: dev cost {c!r} pose {pose.tolist()}")
            print(f"   oracle cost {c2!r} pose {p2.tolist()} iters {it}")
            # the oracle's pose before this iteration and its UpdateCost there
            _, p_prev, _ = O.optimize_scan_match(m, pts, OptimizeScanMatchParam(t - 1, 0.0, 0.0, 0.05, 0.05), init[k])
            e = O.world_to_map(m, p_prev)
            cc, H, bb = O.optimize_update_cost(m, pts, e)
            sx, sy = w.size_x, w.size_y
            cs, sn = np.cos(e[2]), np.sin(e[2])
            x = cs * pts[:, 0] - sn * pts[:, 1] + e[0]
            y = sn * pts[:, 0] + cs * pts[:, 1] + e[1]
            inn = (x > 0) & (x < sx) & (y > 0) & (y < sy)
            print("   est", e.tolist(), "in-map", int(inn.sum()), "of", len(pts),
                  "edge x>sx-1", int((inn & (x > sx - 1)).sum()), "edge y>sy-1", int((inn & (y > sy - 1)).sum()),
                  "x<1", int((inn & (x < 1)).sum()), "y<1", int((inn & (y < 1)).sum()),
                  "integral", int((inn & ((x == np.floor(x)) | (y == np.floor(y)))).sum()))
            bad.append(k)
            break
print("diverging scans:", bad)
