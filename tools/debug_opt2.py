"""Device vs oracle UpdateCost at identical map-cell poses (random and edge)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import pyoracle as O  # noqa: E402
import roborts_csm  # noqa: E402
from roborts_csm import worlds  # noqa: E402

w = worlds.make_world(2000, 2000, 0.05, seed=11)
b = worlds.make_scan_batch(w, 64, seed=12)
ctx = roborts_csm.Context(0)
ctx.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 0), force=True)
m = O.Map(w.grid, w.resolution, w.offset)
rng = np.random.default_rng(1)
nbad = {"cost": 0, "H": 0, "b": 0}
for k in range(64):
    pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
    e0 = O.world_to_map(m, b.init_poses[k])
    for j in range(20):
        e = e0 + rng.normal(size=3) * [2.0, 2.0, 0.05]
        c1, H1, b1 = ctx.optimize_update_cost(pts, e)
        c2, H2, b2 = O.optimize_update_cost(m, pts, e)
        if c1 != c2:
            nbad["cost"] += 1
            if nbad["cost"] <= 5:
                print("cost", k, j, repr(c1), repr(c2), e.tolist())
        nbad["H"] += not np.array_equal(H1, H2)
        nbad["b"] += not np.array_equal(b1, b2)
print("mismatches over", 64 * 20, nbad)
