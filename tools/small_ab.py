"""A/B of the few-window path: single-scan 3-level matches on a 1 cm map
(the reference's shipped fine map), per-kernel HIP-event averages and the
wall p50 per scan. Env knobs are read by the library at csm_create."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "roborts-edu-slam_amd"))
import roborts_csm  # noqa: E402
from roborts_csm import worlds  # noqa: E402
from roborts_csm.params import SIM_YAML_LEVELS  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    w = worlds.make_world(3000, 3000, 0.01, seed=31)
    b = worlds.make_scan_batch(w, 16, seed=5)
    out = {}
    with roborts_csm.Context(0) as ctx:
        ctx.set_grid(roborts_csm.ScanMatchMap(w.grid, 0.01, tuple(w.offset), 0, 1))
        for prof in (False, True):
            ctx.set_profiling(prof)
            lat = []
            for i in range(n):
                k = i % 16
                pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
                pose = np.array(b.init_poses[k])
                cov = np.eye(3).reshape(9).copy()
                t = time.perf_counter()
                ctx.scan_matchers(pts, SIM_YAML_LEVELS, pose, cov)
                lat.append(time.perf_counter() - t)
            lat = np.array(lat[20:]) * 1e3
            if prof:
                out["kernels_us"] = {s["name"]: round(s["total_ms"] / s["launches"] * 1e3, 2)
                                     for s in ctx.kernel_stats() if s["launches"]}
            else:
                out["p50_ms"] = float(np.median(lat))
                out["p10_ms"] = float(np.percentile(lat, 10))
    out["env"] = {k: v for k, v in os.environ.items() if k.startswith("CSM_")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
