"""Which finish mode fails on the headline levels (GPU debug helper)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd")]
import roborts_csm
from roborts_csm import worlds
from roborts_csm.params import headline_levels
w = worlds.make_world(2000, 2000, 0.05)
b = worlds.make_scan_batch(w, 96, seed=99)
for mode in ["exact"] * 6 + [None] * 3:
    if mode:
        os.environ["CSM_FINISH"] = mode
    c = roborts_csm.Context(0)
    os.environ.pop("CSM_FINISH", None)
    c.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 1))
    for prof in (False, True):
        c.set_profiling(prof)
        for li, lv in enumerate(headline_levels()):
            for bs in (8, 96):
                for k0 in range(0, 96, bs):
                    poses = np.ascontiguousarray(b.init_poses[k0:k0 + bs].copy())
                    covs = np.tile(np.eye(3).reshape(1, 9), (bs, 1))
                    try:
                        c.scan_match_batch(b.points_cells[b.offsets[k0]:b.offsets[k0 + bs]],
                                           b.offsets[k0:k0 + bs + 1] - b.offsets[k0], lv, poses, covs)
                    except Exception as e:
                        print(mode, "prof", prof, "level", li, "bs", bs, "scans", k0, "->", e, flush=True)
    c.close()
print("done")
