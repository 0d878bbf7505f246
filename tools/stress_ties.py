"""Stress of the 3-level driver on a map quantised to three values (ties on
every level, so the exact finish pass has windows at every level): the
configuration of tests/test_gpu_parity.py::test_host_signal_split_levels_with_ties,
repeated --iters times in one process against the oracle's answer. Prints one
JSON line: the iterations that differed and, for the first few, the scans and
fields that differ. Run it under the driver's knobs (CSM_HOST_SIGNAL,
CSM_FIRST_WINDOWS, CSM_DEFER_HANDOFF) to see which path an
intermittent mismatch needs.

  python tools/stress_ties.py [--iters 40] [--scans 96]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle")]
os.environ.setdefault("CSM_PIPELINE", "16")
os.environ.setdefault("CSM_PIPELINE_PARTS", "2")
os.environ.setdefault("CSM_FIRST_WINDOWS", "5")
os.environ.setdefault("CSM_SPLIT_HANDOFF_MIN", "8")

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--scans", type=int, default=96)
    ap.add_argument("--seed", type=int, default=99)
    ap.add_argument("--profiling", type=int, default=1, help="HIP-event profiling on, as the test has it")
    a = ap.parse_args()
    import pyoracle as O
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.params import headline_levels
    w = worlds.make_world(2000, 2000, 0.05)
    b = worlds.make_scan_batch(w, a.scans, seed=a.seed)
    grid = np.round(np.asarray(w.grid, dtype=np.float32) * 2.0).astype(np.float32) / np.float32(2.0)
    eye = np.tile(np.eye(3).reshape(1, 9), (b.init_poses.shape[0], 1))
    m = O.Map(grid, w.resolution, w.offset)
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, headline_levels(), b.init_poses, eye.copy())
    c = roborts_csm.Context(0)
    c.set_grid(roborts_csm.ScanMatchMap(grid, float(w.resolution), tuple(w.offset), 0, 1))
    c.set_profiling(bool(a.profiling))
    bad = []
    for it in range(a.iters):
        poses = np.ascontiguousarray(b.init_poses.copy())
        covs = eye.copy()
        s = c.scan_matchers_batch(b.points_cells, b.offsets, headline_levels(), poses, covs)
        ds = np.nonzero(s != s2)[0]
        dp = np.nonzero(np.any(poses != p2, axis=1))[0]
        dc = np.nonzero(np.any(covs != c2, axis=1))[0]
        if ds.size or dp.size or dc.size:
            if len(bad) < 6:
                i = int(np.concatenate([ds, dp, dc])[0])
                bad.append({"iter": it, "scans_score": ds.tolist()[:8], "scans_pose": dp.tolist()[:8],
                            "scans_cov": dc.tolist()[:8], "scan": i, "score": [float(s[i]), float(s2[i])],
                            "pose": [poses[i].tolist(), p2[i].tolist()],
                            "cov_diag": [covs[i][[0, 4, 8]].tolist(), c2[i][[0, 4, 8]].tolist()]})
            else:
                bad.append({"iter": it})
    c.close()
    env = {k: os.environ[k] for k in sorted(os.environ) if k.startswith("CSM_")}
    print(json.dumps({"iters": a.iters, "scans": a.scans, "profiling": a.profiling, "mismatched_iters": len(bad), "env": env,
                      "first": bad[:6]}), flush=True)


if __name__ == "__main__":
    main()
