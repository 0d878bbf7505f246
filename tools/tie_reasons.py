"""Why windows need the exact std::sort pass, on the
CPU: the oracle's scores of every window of the 3-level match at the
bench's configuration, classified with the fast finish's own decisions
(csm_tail.hpp finish(), csm_finish.hip finish_fast_body): which lists each
level keeps (live_lists + own_lists_skip), the FindBest band
|s - best| <= 0.01, the positional set (the first 20 sorted candidates above
min(best - 0.1, 0.5)), the angular set (candidates within the linear
tolerance of FindBest's pose, score >= that bound, first 20). A window is
exact-pass when a tied value (two or more equal scores) sits in the band, at
a positional rank <= 20, or at an angular rank <= 20, or a set exceeds 128.

  python tools/tie_reasons.py [--scans 256] [--levels sim|headline]

Test infrastructure only (imports the oracle)."""
import argparse
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle")]

import pyoracle as O  # noqa: E402
from roborts_csm import worlds, window_dims  # noqa: E402
from roborts_csm.params import COARSE, FINE, SUPER, SIM_YAML_LEVELS, headline_levels  # noqa: E402

KCAP, KCOV = 128, 20


def lists(levels, l):
    """(want_pos, want_ang) of level l: live_lists (csm_driver.cpp) | own_lists_skip (csm_host_finish.cpp)."""
    pos = lambda t: t in (COARSE, FINE)  # noqa: E731 (FAST not used here)
    ang = lambda t: t in (COARSE, SUPER)  # noqa: E731
    skip = 0
    for k in range(l + 1, len(levels)):
        if pos(levels[k].correlation_scan_match_type):
            skip = 3
            break
        if ang(levels[k].correlation_scan_match_type):
            skip |= 2
    skip |= {COARSE: 0, FINE: 2, SUPER: 1}[levels[l].correlation_scan_match_type]
    return not (skip & 1), not (skip & 2)


def classify(sc, na, ns, x0, y0, f, tol, want_pos, want_ang):
    """The reasons (a set) a window goes to the exact pass; empty: the fast path decides it."""
    why = set()
    if np.isnan(sc).any():
        return {"nan"}
    best = sc.max()
    bound = min(best - 0.1, 0.5)
    order = np.argsort(-sc, kind="stable")
    s_sorted = sc[order]
    vals, counts = np.unique(sc, return_counts=True)
    tied = set(vals[counts > 1].tolist())
    band = np.abs(s_sorted - best) <= 1e-2
    if any(v in tied for v in s_sorted[band]):
        why.add("tie in the FindBest band")
    if want_pos:
        above = s_sorted[s_sorted > bound]
        if above.size > KCAP and np.sum(above >= above[min(KCOV, above.size) - 1]) > KCAP:
            why.add("positional set > 128")
        if any(v in tied for v in above[:KCOV + 1]):
            why.add("tie at positional rank <= 20")
    if want_ang:
        nb = int(band.sum())
        idx = order[:nb]
        w = s_sorted[:nb]
        cx = x0 + ((idx // ns) % ns) * f
        cy = y0 + (idx % ns) * f
        bx, by = (np.sum(cx * w) / np.sum(w), np.sum(cy * w) / np.sum(w)) if nb > 1 else (cx[0], cy[0])
        i = np.arange(sc.size)
        near = (np.abs(x0 + ((i // ns) % ns) * f - bx) <= tol) & (np.abs(y0 + (i % ns) * f - by) <= tol) & (sc >= bound)
        nv = np.sort(sc[near])[::-1]
        if nv.size > KCAP:
            why.add("angular set > 128")
        else:  # equal values within the near set (the device counts them there)
            u, cnt = np.unique(nv, return_counts=True)
            tn = set(u[cnt > 1].tolist())
            if any(v in tn for v in nv[:KCOV + 1]):
                why.add("tie at angular rank <= 20")
    return why


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=256)
    ap.add_argument("--levels", choices=["sim", "headline"], default="sim")
    a = ap.parse_args()
    levels = SIM_YAML_LEVELS if a.levels == "sim" else headline_levels()
    world = worlds.make_world(2000, 2000, 0.05, seed=20261015)
    batch = worlds.make_scan_batch(world, a.scans, seed=1000)  # bench.py's rank-0 batch
    m = O.Map(world.grid, world.resolution, world.offset)
    O.set_threads(min(16, os.cpu_count() or 1))
    stats = [collections.Counter() for _ in levels]
    for k in range(a.scans):
        pts = batch.points_cells[batch.offsets[k]:batch.offsets[k + 1]]
        pose, cov = batch.init_poses[k].copy(), np.eye(3)
        for l, p in enumerate(levels):
            na, ns = window_dims(p)
            c = O.world_to_map(m, pose)
            sc = O.score_window(m, pts, p, c, na * ns * ns)
            f = p.search_space_resolution / world.resolution
            x0 = c[0] - (p.search_space_size / world.resolution) * 0.5
            y0 = c[1] - (p.search_space_size / world.resolution) * 0.5
            wp, wa = lists(levels, l)
            why = classify(sc, na, ns, x0, y0, f, f, wp, wa)
            stats[l]["windows"] += 1
            stats[l]["exact"] += bool(why)
            for r in why:
                stats[l][r] += 1
            _, pose, cov, _, _ = O.scan_match(m, pts, p, pose, cov)
    for l, s in enumerate(levels):
        na, ns = window_dims(s)
        st = stats[l]
        print(f"level {l} ({na}x{ns}^2 = {na * ns * ns} candidates, lists pos/ang {lists(levels, l)}): "
              f"{st['exact']} of {st['windows']} windows exact ({100 * st['exact'] / st['windows']:.1f} %)")
        for r, n in st.most_common():
            if r not in ("windows", "exact"):
                print(f"    {r:32s} {n:5d}")


if __name__ == "__main__":
    main()
