"""Design statistics for the coarse box kernel (CPU, numpy): over config 2's
scans and the coarse level's 30 angles, the run lists (consecutive beams with
one box corner), their count distribution, how many equal-count pairs a
count-sorted list forms per 576-beam segment, and the 128-byte cache lines a
run's 13 box rows touch under three layouts of the one-byte palette grid:
row-major (pitch 2016 B), and column strips of 16 or 32 bytes (rows of a strip
contiguous) with 4 or 2 byte-shifted copies so every 16-byte row piece sits in
one strip row.

  python tools/box_layout_stats.py [n_scans]
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd")]

import numpy as np  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    from roborts_csm import worlds
    w = worlds.make_world(2000, 2000, 0.05)
    b = worlds.make_scan_batch(w, n, seed=7)
    ns, na, seg = 13, 30, 576
    angles = -0.523 + 0.0349 * np.arange(na) + 0.0349 / 2 * 0  # spacing is what matters here
    pitch = 2016
    cnt_hist = np.zeros(1100, np.int64)
    runs_tot = pairs_tot = 0
    lines = {"rowmajor": 0, "strip16x4": 0, "strip32x2": 0}
    waves = 0
    for s in range(n):
        p = b.points_cells[b.offsets[s]:b.offsets[s + 1]]
        px, py, th = b.init_poses[s]
        cx, cy = px / w.resolution, py / w.resolution
        for a in angles:
            c, si = math.cos(th + a), math.sin(th + a)
            lx = c * p[:, 0] - si * p[:, 1]
            ly = si * p[:, 0] + c * p[:, 1]
            ix = np.trunc(lx + (cx - 6) + 0.5).astype(np.int64)
            iy = np.trunc(ly + (cy - 6) + 0.5).astype(np.int64)
            waves += 1
            for s0 in range(0, len(ix), seg):
                kx, ky = ix[s0:s0 + seg], iy[s0:s0 + seg]
                edge = np.ones(len(kx), bool)
                edge[1:] = (kx[1:] != kx[:-1]) | (ky[1:] != ky[:-1])
                st = np.nonzero(edge)[0]
                cn = np.diff(np.append(st, len(kx)))
                rx, ry = kx[st], ky[st]
                runs_tot += len(st)
                np.add.at(cnt_hist, cn, 1)
                _, per = np.unique(cn, return_counts=True)
                pairs_tot += int(np.sum((per + 1) // 2))
                k = np.arange(ns)[None, :]
                y = ry[:, None] + k
                # row-major: 16 bytes at (x & ~3) of each row
                a0 = y * pitch + (rx[:, None] & ~3)
                l0 = a0 // 128
                l1 = (a0 + 15) // 128
                lines["rowmajor"] += int(np.sum(l0 != l1) + l0.size)
                # strips of width W: copy chosen so the piece fits one strip row; per run,
                # rows contiguous at W bytes: lines = distinct (y*W)//128 (+ second line if a
                # piece straddles, impossible here)
                for name, W in (("strip16x4", 16), ("strip32x2", 32)):
                    off = y * W
                    ln = off // 128
                    lines[name] += int(np.sum(ln[:, 1:] != ln[:, :-1]) + ln.shape[0])
    print(f"scans {n}, waves {waves}: runs/wave {runs_tot / waves:.1f}, "
          f"equal-count pairs/wave {pairs_tot / waves:.1f} ({pairs_tot / runs_tot:.3f} per run)")
    top = np.argsort(-cnt_hist)[:12]
    print("run count histogram (count: share):",
          ", ".join(f"{c}: {cnt_hist[c] / runs_tot:.3f}" for c in top if cnt_hist[c]))
    for k, v in lines.items():
        print(f"  {k:10s} lines per run {v / runs_tot:.2f}")


if __name__ == "__main__":
    main()
