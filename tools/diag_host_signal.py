"""Diagnostic: repeat test_host_signal_finish_repeated's configuration (96
scans, 3 headline levels, CSM_PIPELINE=16, CSM_FIRST_WINDOWS=8, host-signal
finish) many times and report every mismatch against the oracle: which scan,
which covariance entries, the values, and whether the wrong value equals the
answer of the scan's previous batch position or level (stale records).

  python tools/diag_host_signal.py [iterations] [ENV=VALUE ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    env = {"CSM_PIPELINE": "16", "CSM_HOST_SIGNAL": "1", "CSM_FIRST_WINDOWS": "8"}
    for a in sys.argv[2:]:
        k, v = a.split("=", 1)
        env[k] = v
    os.environ.update(env)
    import pyoracle as O
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.params import headline_levels
    w = worlds.make_world(2000, 2000, 0.05)
    b = worlds.make_scan_batch(w, 96, seed=99)
    m = O.Map(w.grid, w.resolution, w.offset)
    eye = np.tile(np.eye(3).reshape(1, 9), (b.init_poses.shape[0], 1))
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, headline_levels(), b.init_poses, eye.copy())
    c = roborts_csm.Context(0)
    c.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 1))
    c.load_scans(b.points_cells, b.offsets)
    bad = 0
    for it in range(iters):
        poses = np.ascontiguousarray(b.init_poses.copy())
        covs = eye.copy()
        s = c.scan_matchers_loaded(headline_levels(), poses, covs)
        ok_s, ok_p, ok_c = np.array_equal(s, s2), np.array_equal(poses, p2), np.array_equal(covs, c2)
        if ok_s and ok_p and ok_c:
            continue
        bad += 1
        rows = sorted(set(np.nonzero((s != s2) | (poses != p2).any(1) | (covs != c2).any(1))[0].tolist()))
        print(f"iter {it}: scores {ok_s} poses {ok_p} covs {ok_c}; scans {rows}", flush=True)
        for r in rows[:6]:
            d = np.nonzero(covs[r] != c2[r])[0].tolist()
            print(f"  scan {r} (part {r // 48}, window {r % 48}): cov entries {d} got {covs[r][d]} want {c2[r][d]}"
                  f" | score {s[r]!r} vs {s2[r]!r} | pose {poses[r]} vs {p2[r]}", flush=True)
    print(f"{bad} of {iters} batches differ ({env})", flush=True)
    c.close()


if __name__ == "__main__":
    main()
