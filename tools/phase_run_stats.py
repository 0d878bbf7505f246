# Run statistics of the fine level's phase kernel on config 2: per (window,
# angle), beams whose (box corner, bucket pair) equals the previous beam's in
# the same pair list (so one box load could serve both, times the run length).
# Host-only numpy, seeded config-2 world and scans; phase buckets from the
# library's own table (csm_api.cpp phase_table, restated here in float64 with
# the same breakpoints). Usage: python tools/phase_run_stats.py [scans]
import math
import sys

import numpy as np

sys.path[:0] = ['roborts-edu-slam_amd']
from roborts_csm import worlds  # noqa: E402
from roborts_csm.params import headline_levels  # noqa: E402

lv = headline_levels()[1]
w = worlds.make_world(2000, 2000, 0.05, seed=20261015)
n_scans = int(sys.argv[1]) if len(sys.argv) > 1 else 8
b = worlds.make_scan_batch(w, n_scans, seed=1000)
res = w.resolution
f = lv.search_space_resolution / res
ns = int(round(lv.search_space_size / lv.search_space_resolution)) + 1
# breakpoints ceil(j f) - j f: bucket = index of the gap a phase falls in
bp = sorted({0.0, 1.0} | {math.ceil(j * f) - j * f for j in range(ns)})
bp = np.array(bp)


def bucket(ph):
    return np.searchsorted(bp, ph, side="right") - 1


tot_beams = tot_runs = tot_keys = tot_adj = 0
for k in range(n_scans):
    pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
    pose = b.init_poses[k]
    s = 1 / res
    cx, cy = s * pose[0] + s * w.offset[0], s * pose[1] + s * w.offset[1]
    x0 = cx - (lv.search_space_size / res) * 0.5
    y0 = cy - (lv.search_space_size / res) * 0.5
    na = int(math.floor(2 * lv.search_angle_offset / lv.search_angle_resolution)) + 1
    for a in range(na):
        th = pose[2] - lv.search_angle_offset + a * lv.search_angle_resolution
        c, sn = math.cos(th), math.sin(th)
        lx = c * pts[:, 0] - sn * pts[:, 1]
        ly = sn * pts[:, 0] + c * pts[:, 1]
        tx, ty = (lx + x0) + 0.5, (ly + y0) + 0.5
        X, Y = np.floor(tx).astype(np.int64), np.floor(ty).astype(np.int64)
        qx, qy = bucket(tx - X), bucket(ty - Y)
        key = ((X * 100003 + Y) * 64 + qx * 8 + qy)
        pair = qx * 8 + qy
        tot_beams += len(key)
        tot_keys += len(np.unique(key))
        # runs inside each pair list (beam order within a pair)
        runs = 0
        for p in np.unique(pair):
            kk = key[pair == p]
            runs += 1 + int(np.count_nonzero(kk[1:] != kk[:-1]))
        tot_runs += runs
        # runs of adjacent beams (consecutive in beam order)
        tot_adj += 1 + int(np.count_nonzero(key[1:] != key[:-1]))
print(f"fine level f={f:.3f} ns={ns}: beams per (window, angle) {tot_beams / (n_scans * na):.0f}")
print(f"  distinct (corner, pair) keys      {tot_keys / tot_beams:.3f} per beam")
print(f"  runs inside pair lists             {tot_runs / tot_beams:.3f} per beam")
print(f"  runs of adjacent beams             {tot_adj / tot_beams:.3f} per beam")
