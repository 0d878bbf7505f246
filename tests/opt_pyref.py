"""Independent pure-Python restatement of the Gauss-Newton scan matcher
(optimize_scan_matcher.h:68-221), used to pin oracle/opt_oracle.cpp.

Written from the reference's expressions, not from the oracle's source:
Python floats are IEEE doubles and every operation below is evaluated in the
reference's order (no FMA), so results compare bit for bit. Slow (one Python
loop per point): small cases only.
"""
from __future__ import annotations

import math

import numpy as np

from libm import sincos

K_COST_POINT_SIZE = 1000.0   # optimize_scan_matcher.h:234
K_MAX_COST = 1.0 * K_COST_POINT_SIZE


def _cell(grid, x, y, outside):
    sy, sx = grid.shape
    idx = y * sx + x
    if idx < 0 or idx >= sx * sy:
        return float(np.float32(outside))
    return float(grid.reshape(-1)[idx])


def update_cost(grid, pts, est, outside=0.3):
    """UpdateCost (:154-221) -> (cost, H 3x3 list, b list)."""
    sy, sx = grid.shape
    c, s = sincos(est[2])  # GCC merges the cos/sin pairs of :96-97,:200-201 into sincos
    H = [[0.0] * 3 for _ in range(3)]
    b = [0.0] * 3
    cost = 0.0
    valid = 1
    for lx, ly in pts:
        lx, ly = float(lx), float(ly)
        x = (c * lx + (-s) * ly) + est[0]
        y = (s * lx + c * ly) + est[1]
        if not (x > 0 and x < sx and y > 0 and y < sy):
            continue
        x0, y0, x1, y1 = math.floor(x), math.floor(y), math.ceil(x), math.ceil(y)
        p00 = _cell(grid, int(x0), int(y0), outside)
        p01 = _cell(grid, int(x0), int(y1), outside)
        p10 = _cell(grid, int(x1), int(y0), outside)
        p11 = _cell(grid, int(x1), int(y1), outside)
        x0, y0, x1, y1 = float(x0), float(y0), float(x1), float(y1)
        r = (y - y0) * (p11 * (x - x0) + p01 * (x1 - x)) + (y1 - y) * (p10 * (x - x0) + p00 * (x1 - x))
        r = (r if r <= 1 else 1.0) if r >= 0 else 0.0
        e = 1 - r
        cost += e * e
        ds = ((-s) * lx - c * ly, c * lx - s * ly)
        dm0 = (y - y0) * (p11 - p01) + (y1 - y) * (p10 - p00)
        dm1 = (x - x0) * (p11 - p10) + (x1 - x) * (p01 - p00)
        n0, n1 = -dm0, -dm1
        J = (n0 * 1.0 + n1 * 0.0, n0 * 0.0 + n1 * 1.0, n0 * ds[0] + n1 * ds[1])
        for i in range(3):
            for j in range(3):
                H[i][j] += J[i] * J[j]
        for i in range(3):
            b[i] += (-J[i]) * e
        valid += 1
    cost *= K_COST_POINT_SIZE / valid
    return cost, H, b


def ldlt_solve(H, b):
    """Eigen 3.3 LDLT<Matrix3d, Lower>::solve."""
    a = [[float(H[i][j]) for j in range(3)] for i in range(3)]
    tr = [0, 1, 2]
    for k in range(3):
        big = k
        for i in range(k + 1, 3):
            if abs(a[i][i]) > abs(a[big][big]):
                big = i
        tr[k] = big
        if big != k:
            for j in range(k):
                a[k][j], a[big][j] = a[big][j], a[k][j]
            for i in range(big + 1, 3):
                a[i][k], a[i][big] = a[i][big], a[i][k]
            a[k][k], a[big][big] = a[big][big], a[k][k]
            for i in range(k + 1, big):
                a[i][k], a[big][i] = a[big][i], a[i][k]
        if k > 0:
            t = [a[i][i] * a[k][i] for i in range(k)]
            d = a[k][0] * t[0] if k == 1 else a[k][0] * t[0] + a[k][1] * t[1]
            a[k][k] -= d
            if k == 1:
                a[2][1] -= a[2][0] * t[0]
        akk = a[k][k]
        if k == 0 and not abs(akk) > 0:
            tr = [0, 1, 2]
            break
        if k < 2 and abs(akk) > 0:
            for r in range(k + 1, 3):
                a[r][k] /= akk
    d = [float(v) for v in b]
    for k in range(3):
        d[k], d[tr[k]] = d[tr[k]], d[k]
    d[1] -= a[1][0] * d[0]
    d[2] -= a[2][0] * d[0] + a[2][1] * d[1]
    tiny = np.finfo(np.float64).tiny
    for i in range(3):
        d[i] = d[i] / a[i][i] if abs(a[i][i]) > tiny else 0.0
    d[1] -= a[2][1] * d[2]
    d[0] -= a[1][0] * d[1] + a[2][0] * d[2]
    for k in (2, 1, 0):
        d[k], d[tr[k]] = d[tr[k]], d[k]
    return d


def _limit(v, lim):  # util::MaxAbxLimit
    if v > abs(lim):
        return abs(lim)
    if v < -abs(lim):
        return -abs(lim)
    return v


def _normalize(a):  # util::NormalizeAngle
    n = math.fmod(math.fmod(a, 2.0 * math.pi) + 2.0 * math.pi, 2.0 * math.pi)
    return n - 2.0 * math.pi if n > math.pi else n


def optimize_scan_match(grid, resolution, offset, pts, param, pose, map_init=True, outside=0.3):
    """BasedOptimizeScanMatch::ScanMatch -> (cost, pose', iterations)."""
    pose = [float(v) for v in pose]
    if not map_init or len(pts) == 0:
        return K_MAX_COST, pose, 0
    sf = 1.0 / resolution
    est = [sf * pose[0] + sf * offset[0], sf * pose[1] + sf * offset[1], pose[2]]
    mres = 1 / sf
    cost = 0.0
    its = 0
    for it in range(int(param.iterate_max_times)):
        last = cost
        cost, H, b = update_cost(grid, pts, est, outside)
        its = it + 1
        det = ldlt_solve(H, b)
        if any(math.isnan(v) for v in det):
            return K_MAX_COST, pose, its
        if it > 0 and (last - cost < param.cost_decrease_threshold or cost < param.cost_min_threshold):
            break
        est[0] += _limit(det[0], param.max_update_distance / mres)
        est[1] += _limit(det[1], param.max_update_distance / mres)
        est[2] += _limit(det[2], param.max_update_angle)
    est[2] = _normalize(est[2])
    tx, ty = sf * offset[0], sf * offset[1]
    a = sf * (1.0 / (sf * sf - 0.0 * 0.0))
    return cost, [a * est[0] + (-(a * tx)), a * est[1] + (-(a * ty)), est[2]], its
