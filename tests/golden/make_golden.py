"""Generate the committed golden fixtures tests/golden/*.npz.

PARITY UNPINNED: the reference holds no golden vectors for this path and can
not be compiled here, so the expected outputs come from the CPU
oracle (oracle/csm_oracle.cpp, a line-by-line restatement of the reference).
These fixtures pin the oracle against regressions and give the GPU parity tests
fixed inputs; tests/test_oracle_golden.py also cross-checks them against the
independent pure-Python restatement in tests/pyref.py.

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle")]

import pyoracle as O  # noqa: E402
from roborts_csm import worlds  # noqa: E402
from roborts_csm.params import (  # noqa: E402
    CONFIG1_PARAM, FAST_PARAM, PARAM_CONFIG_LEVELS, PARAM_CONFIG_OPTIMIZE, SIM_YAML_LEVELS, SIM_YAML_OPTIMIZE,
    CorrelationScanMatchParam, headline_levels,
)

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 20261015


def _param_arr(p) -> np.ndarray:
    return np.array([p.search_space_size, p.search_space_resolution, p.search_angle_offset,
                     p.search_angle_resolution, p.response_threshold, p.use_point_size, p.max_depth,
                     int(p.use_center_penalty), p.correlation_scan_match_type], dtype=np.float64)


def dims(p):
    half = (p.search_angle_offset * 2) / 2
    na = int(math.floor(half * 2 / p.search_angle_resolution) + 1)
    v = p.search_space_size / p.search_space_resolution
    ns = int((math.floor(v + 0.5) if v >= 0 else math.ceil(v - 0.5)) + 1)
    return na, ns


def crop(world, cx, cy, size):
    """size x size crop centred on cell (cx, cy) with the matching map offset."""
    x0, y0 = int(cx) - size // 2, int(cy) - size // 2
    g = np.ascontiguousarray(world.grid[y0:y0 + size, x0:x0 + size])
    # world_to_map(w) = (w + off)/res; crop shifts cells by (x0, y0)
    off = (world.offset[0] - x0 * world.resolution, world.offset[1] - y0 * world.resolution)
    return g, off


def level_trace(m, pts, levels, pose0):
    """Per-level centre, all scores and sorted order of the 3-level driver."""
    pose = np.array(pose0, dtype=np.float64)
    cov = np.eye(3).reshape(9)
    out = {}
    for li, p in enumerate(levels):
        na, ns = dims(p)
        c = O.world_to_map(m, pose)
        out[f"l{li}_center"] = c
        out[f"l{li}_scores"] = O.score_window(m, pts, p, c, na * ns * ns)
        out[f"l{li}_order"] = O.sorted_order(m, pts, p, c, na * ns * ns)
        r, pose, cov, am, _ = O.scan_match(m, pts, p, pose, cov)
        out[f"l{li}_response"] = np.float64(r)
        out[f"l{li}_pose"] = pose.copy()
        out[f"l{li}_cov"] = cov.copy()
        out[f"l{li}_argmax"] = np.int64(am)
    return out


def gen_config1():
    """F1: BASELINE config 1 — 361-beam scan, 400x400 @5 cm, +-0.5 m / +-15 deg."""
    w = worlds.make_world(400, 400, 0.05, seed=SEED)
    laser = worlds.LaserSpec(n_beams=361, fov_deg=180.0)
    b = worlds.make_scan_batch(w, 1, seed=SEED + 1, laser=laser)
    pts = b.points_cells
    m = O.Map(w.grid, w.resolution, w.offset)
    p = CONFIG1_PARAM
    na, ns = dims(p)
    c = O.world_to_map(m, b.init_poses[0])
    scores = O.score_window(m, pts, p, c, na * ns * ns)
    order = O.sorted_order(m, pts, p, c, na * ns * ns)
    r, pose, cov, am, _ = O.scan_match(m, pts, p, b.init_poses[0], np.eye(3))
    r3, pose3, cov3 = O.scan_matchers(m, pts, SIM_YAML_LEVELS, b.init_poses[0], np.eye(3))
    np.savez_compressed(os.path.join(OUT, "f1_config1.npz"), grid=w.grid, resolution=w.resolution,
                        offset=np.array(w.offset), points=pts, init_pose=b.init_poses[0],
                        true_pose=b.true_poses[0], param=_param_arr(p), center=c, scores=scores,
                        order=order, response=r, pose=pose, cov=cov, argmax=am,
                        sim3_score=r3, sim3_pose=pose3, sim3_cov=cov3)
    print("f1", na * ns * ns, "candidates, response", r, "argmax", am)


def gen_config2_crop():
    """F2: 1081-beam scan on a 600x600 crop of the 2000x2000 world, 3 levels
    (SIM YAML, U=100 -> B=109) and the headline B=1081 variant."""
    w = worlds.make_world(2000, 2000, 0.05, seed=SEED)
    b = worlds.make_scan_batch(w, 4, seed=SEED + 2)
    k = 0
    tp = b.true_poses[k]
    cx, cy = (tp[0] + w.offset[0]) / w.resolution, (tp[1] + w.offset[1]) / w.resolution
    g, off = crop(w, cx, cy, 600)
    m = O.Map(g, w.resolution, off)
    pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
    d = {"grid": g, "resolution": w.resolution, "offset": np.array(off), "points": pts,
         "init_pose": b.init_poses[k], "true_pose": tp}
    for tag, levels in (("sim", SIM_YAML_LEVELS), ("b1081", headline_levels()),
                        ("pcfg", PARAM_CONFIG_LEVELS)):
        tr = level_trace(m, pts, levels, b.init_poses[k])
        d.update({f"{tag}_{kk}": v for kk, v in tr.items()})
        s, pose, cov = O.scan_matchers(m, pts, levels, b.init_poses[k], np.eye(3))
        d[f"{tag}_score"] = s
        d[f"{tag}_pose"] = pose
        d[f"{tag}_cov"] = cov
        d[f"{tag}_levels"] = np.stack([_param_arr(l) for l in levels])
        print("f2", tag, "score", s, "pose err", pose - tp)
    np.savez_compressed(os.path.join(OUT, "f2_config2_crop.npz"), **d)


def gen_ties():
    """F3: a flat region where whole groups of candidates tie exactly, to pin
    std::sort's tie order (the reference sorts with std::sort, :607)."""
    g = np.full((200, 200), np.float32(0.3), dtype=np.float32)
    g[150:153, 20:180] = np.float32(1.0)  # one far wall only some beams reach
    g[20:180, 170:172] = np.float32(0.7)
    rng = np.random.default_rng(SEED + 3)
    ang = rng.uniform(-math.pi, math.pi, 300)
    rad = rng.uniform(5, 60, 300)
    pts = np.stack([np.cos(ang) * rad, np.sin(ang) * rad], axis=1)
    m = O.Map(g, 0.05, (5.0, 5.0))
    init = np.array([0.02, -0.01, 0.1])
    out = {"grid": g, "resolution": 0.05, "offset": np.array([5.0, 5.0]), "points": pts, "init_pose": init}
    for tag, p in (("pen", CONFIG1_PARAM), ("nopen", CONFIG1_PARAM.with_(use_center_penalty=False)),
                   ("fine", SIM_YAML_LEVELS[1].with_(use_center_penalty=False))):
        na, ns = dims(p)
        c = O.world_to_map(m, init)
        out[f"{tag}_param"] = _param_arr(p)
        out[f"{tag}_scores"] = O.score_window(m, pts, p, c, na * ns * ns)
        out[f"{tag}_order"] = O.sorted_order(m, pts, p, c, na * ns * ns)
        r, pose, cov, am, _ = O.scan_match(m, pts, p, init, np.eye(3))
        out[f"{tag}_response"] = r
        out[f"{tag}_pose"] = pose
        out[f"{tag}_cov"] = cov
        out[f"{tag}_argmax"] = am
        nt = len(np.unique(out[f"{tag}_scores"]))
        print("f3", tag, "unique scores", nt, "of", na * ns * ns)
    np.savez_compressed(os.path.join(OUT, "f3_ties.npz"), **out)


def gen_bnb():
    """F4: the reference's dormant branch-and-bound (FAST) on the F1 inputs."""
    f1 = np.load(os.path.join(OUT, "f1_config1.npz"))
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    r, pose, cov, _, nsc = O.scan_match(m, f1["points"], FAST_PARAM, f1["init_pose"], np.eye(3))
    np.savez_compressed(os.path.join(OUT, "f4_bnb.npz"), param=_param_arr(FAST_PARAM), response=r,
                        pose=pose, cov=cov, n_scored=nsc)
    print("f4 bnb response", r, "scored", nsc)


def gen_large_window():
    """F5: argmax-only, +-2 m / +-180 deg window on the F1 grid (loop-closure shape)."""
    f1 = np.load(os.path.join(OUT, "f1_config1.npz"))
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    p = CorrelationScanMatchParam(4.0, 0.05, math.pi, 0.0349, 0.5, 100, 0, False, 0)
    c = O.world_to_map(m, f1["init_pose"])
    s, flat = O.best_window(m, f1["points"], p, c)
    np.savez_compressed(os.path.join(OUT, "f5_large_window.npz"), param=_param_arr(p), center=c,
                        best_score=s, best_flat=flat)
    print("f5 best", s, flat)


def gen_optimize():
    """F6: the Gauss-Newton matcher (optimize_scan_matcher.h:68-132) on the F1
    grid: the F1 scan plus 5 ray-cast scans, both reference parameter sets
    (simulatin_param.yaml:42-47 and ParamConfig defaults param_config.h:63-69)."""
    f1 = np.load(os.path.join(OUT, "f1_config1.npz"))
    res, off = float(f1["resolution"]), tuple(f1["offset"])
    m = O.Map(f1["grid"], res, off)
    w = worlds.World(f1["grid"], f1["grid"] >= 0.99, res, off)
    b = worlds.make_scan_batch(w, 5, seed=SEED + 6)
    pts = [f1["points"]] + [b.points_cells[b.offsets[k]:b.offsets[k + 1]] for k in range(5)]
    init = np.vstack([f1["init_pose"], b.init_poses])
    offsets = np.concatenate([[0], np.cumsum([len(p) for p in pts])]).astype(np.int64)
    out = {"points": np.vstack(pts), "offsets": offsets, "init_poses": init}
    for tag, prm in (("sim", SIM_YAML_OPTIMIZE), ("cfg", PARAM_CONFIG_OPTIMIZE)):
        out[f"param_{tag}"] = np.array([prm.iterate_max_times, prm.cost_decrease_threshold, prm.cost_min_threshold,
                                        prm.max_update_distance, prm.max_update_angle])
        r = [O.optimize_scan_match(m, p, prm, q) for p, q in zip(pts, init)]
        out[f"cost_{tag}"] = np.array([x[0] for x in r])
        out[f"pose_{tag}"] = np.vstack([x[1] for x in r])
        out[f"iters_{tag}"] = np.array([x[2] for x in r], dtype=np.int32)
        print("f6", tag, "costs", np.round(out[f"cost_{tag}"], 3), "iters", out[f"iters_{tag}"])
    np.savez_compressed(os.path.join(OUT, "f6_optimize.npz"), **out)


GENERATORS = {"f1": gen_config1, "f2": gen_config2_crop, "f3": gen_ties, "f4": gen_bnb, "f5": gen_large_window,
              "f6": gen_optimize}

if __name__ == "__main__":
    # python tests/golden/make_golden.py [f1 f2 ...]  (default: all, in order)
    for name in (sys.argv[1:] or list(GENERATORS)):
        GENERATORS[name]()
