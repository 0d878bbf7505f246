"""Independent numpy restatement of the reference scan matcher (test-only).

A second, separately written restatement used to cross-check the C++ oracle
on the golden fixtures: vectorised over candidates, sequential over beams (so
the fp64 sums round exactly as the reference's per-candidate loop), the
candidate sort done by the pure-Python libstdc++ introsort model.
Citations: correlate_scan_matcher.h unless noted.
"""
from __future__ import annotations

import math

import numpy as np

from introsort_ref import sort_order_greater
from libm import sincos


def dims(p):
    half = (p.search_angle_offset * 2) / 2                        # :526,:536
    na = int(math.floor(half * 2 / p.search_angle_resolution) + 1)  # :154
    v = p.search_space_size / p.search_space_resolution
    ns = int((math.floor(v + 0.5) if v >= 0 else math.ceil(v - 0.5)) + 1)  # :538
    return na, ns


def window_scores(grid: np.ndarray, pts: np.ndarray, p, center, mres: float, outside=np.float32(0.3)):
    """Penalised scores of every candidate, enumeration order (theta, x, y)."""
    na, ns = dims(p)
    n = pts.shape[0]
    use = int(p.use_point_size)
    if n < 2 * use:                                               # :561-566
        use, step = n, 1
    else:
        step = n // (use - 1)
    half = (p.search_angle_offset * 2) / 2
    start = center[2] - half
    angles = np.array([start + a * p.search_angle_resolution for a in range(na)])
    x0 = center[0] - (p.search_space_size / mres) * 0.5           # :546
    y0 = center[1] - (p.search_space_size / mres) * 0.5
    f = p.search_space_resolution / mres
    xs = x0 + np.arange(ns) * f                                   # :569
    ys = y0 + np.arange(ns) * f                                   # :572
    H, W = grid.shape
    out = np.empty((na, ns, ns))
    for a in range(na):
        c, s = sincos(angles[a])                                 # :171-172 (GCC: one sincos)
        acc = np.zeros((ns, ns))
        for q in range(0, n, step):                               # :645
            px, py = pts[q, 0], pts[q, 1]
            lx = c * px - s * py                                  # :179
            ly = s * px + c * py                                  # :180
            gx = np.trunc((lx + xs) + 0.5).astype(np.int64)       # :647
            gy = np.trunc((ly + ys) + 0.5).astype(np.int64)       # :648
            ok = (gx[:, None] >= 0) & (gx[:, None] < W) & (gy[None, :] >= 0) & (gy[None, :] < H)
            v = grid[np.clip(gy[None, :], 0, H - 1), np.clip(gx[:, None], 0, W - 1)]
            acc = acc + np.where(ok, v, outside).astype(np.float64)
        out[a] = acc / use                                        # :659
    sc = out.reshape(-1)
    if p.use_center_penalty:                                      # :587-603, :718-745
        g = 0.4 if p.correlation_scan_match_type == 0 else 0.2
        A = np.repeat(angles, ns * ns)
        X = np.tile(np.repeat(xs, ns), na)
        Y = np.tile(ys, na * ns)
        dx, dy = X - center[0], Y - center[1]
        d2 = (dx * dx + dy * dy) * (mres * mres)
        dp = np.maximum(1.0 - (g * d2 / (p.search_space_size / 2)), 0.5)
        da = (A - center[2]) ** 2
        ap = np.maximum(1.0 - (0.25 * da / 0.349), 0.9)
        zero = np.abs(sc) <= 1e-06
        sc = np.where(zero, sc, sc * (dp * ap))
    return sc, angles, xs, ys


def sorted_order(scores) -> np.ndarray:
    return np.array(sort_order_greater(scores), dtype=np.int64)
