"""Independent pure-Python restatement of the reference's map building
(map/occu_grid_map.h, map/grid_map_base.h, map/grid_map_cell.h,
util/boundbox.h), written separately from oracle/map_oracle.cpp to pin it on
small cases (test infrastructure; the reference has no map tests and cannot
be compiled here). float32 cell arithmetic uses numpy float32 scalars, which
round like the reference's float operations.
"""
from __future__ import annotations

import math

import numpy as np

from libm import sincos

F = np.float32
FLT_MAX = float(np.finfo(np.float32).max)
FLT_MIN = float(np.finfo(np.float32).tiny)


def bresenham(x0, y0, x1, y1):
    """LineVisitor::ErgodLineBresenhami (occu_grid_map.h:125-188)."""
    steep = abs(y1 - y0) > abs(x1 - x0)
    if steep:
        x0, y0, x1, y1 = y0, x0, y1, x1
    if x0 > x1:
        x0, x1, y0, y1 = x1, x0, y1, y0
    dx, dy = x1 - x0, abs(y1 - y0)
    err, y = 0, y0
    ys = 1 if y0 < y1 else -1
    out = []
    for x in range(x0, x1 + 1):
        out.append((y, x) if steep else (x, y))
        err += dy
        if 2 * err >= dx:
            y += ys
            err -= dx
    return out


def bresenham_closed_form(x0, y0, x1, y1):
    """The kernels' closed form of the same walk (csm_gridmap.hip, Line::at)."""
    steep = abs(y1 - y0) > abs(x1 - x0)
    if steep:
        x0, y0, x1, y1 = y0, x0, y1, x1
    if x0 > x1:
        x0, x1, y0, y1 = x1, x0, y1, y0
    dx, dy = x1 - x0, abs(y1 - y0)
    ys = 1 if y0 < y1 else -1
    out = []
    for t in range(dx + 1):
        c = (2 * t * dy + dx) // (2 * dx) if dx else 0
        X, Y = x0 + t, y0 + ys * c
        out.append((Y, X) if steep else (X, Y))
    return out


class PyMap:
    def __init__(self, kind, res, size, off, deviation=0.0, default_prob=0.5):
        self.kind = kind  # 0 probability, 1 count
        self.s = 1.0 / res
        self.sx, self.sy = int(size[0]), int(size[1])
        self.row = self.sx
        self.ox, self.oy = float(off[0]), float(off[1])
        self.bmin = [FLT_MAX, FLT_MAX]
        self.bmax = [FLT_MIN, FLT_MIN]
        self.ext = 1.0
        self.dflt = F(default_prob)
        self.mui = -1
        n = self.sx * self.sy
        # new CellType[n]{default}: element 0 from default, the rest 0.5f
        self.prob = [F(0.5)] * n
        if n:
            self.prob[0] = self.dflt
        self.pas = [F(0.0)] * n
        self.hit = [F(0.0)] * n
        self.uidx = [-1] * n
        if deviation > 0.5 * res and deviation < 10 * res and res > 0:
            self.blur_ok = True
            self.hk = int((deviation / res) * math.sqrt(math.log(2)))
            ks = 2 * self.hk + 1
            self.kern = [0.0] * (ks * ks)
            for i in range(-self.hk, self.hk + 1):
                for j in range(-self.hk, self.hk + 1):
                    d = math.hypot(i * res, j * res)
                    q = d / deviation
                    self.kern[(i + self.hk) + ks * (j + self.hk)] = math.exp(-0.5 * (q * q))
        else:
            self.blur_ok, self.hk, self.kern = False, 0, []
        self.auto, self.just = True, False
        self.cur, self.cf, self.co = 0, -1, -1
        self.offs = 0.72
        self.points = []
        if kind == 1:
            self.ff, self.fo, self.thr, self.mp = F(0), F(0), F(0.5), F(2)
        else:
            self.ff, self.fo, self.thr, self.mp = F(0.2), F(0.5), F(0.5), F(2)

    # cell functions
    def occ(self, i):
        if self.kind == 1:
            self.hit[i] = F(self.hit[i] + F(F(1) + self.fo))
            self.pas[i] = F(self.pas[i] + F(F(1) + self.ff))
            with np.errstate(divide="ignore", invalid="ignore"):
                v = F(self.hit[i] / self.pas[i])
            self.prob[i] = F(1) if v > F(1) else v
        else:
            v = F(self.prob[i] + self.fo)
            self.prob[i] = F(1) if v > F(1) else v

    def free(self, i):
        if self.kind == 1:
            self.pas[i] = F(self.pas[i] + F(F(1) + self.ff))
            with np.errstate(divide="ignore", invalid="ignore"):
                self.prob[i] = F(self.hit[i] / self.pas[i])
        else:
            v = F(self.prob[i] - self.ff)
            self.prob[i] = F(0) if v < F(0) else v

    def unfree(self, i):
        if self.kind == 1:
            self.pas[i] = F(self.pas[i] - F(F(1) + self.ff))
            with np.errstate(divide="ignore", invalid="ignore"):
                self.prob[i] = F(self.hit[i] / self.pas[i])
        else:
            v = F(self.prob[i] + self.ff)
            self.prob[i] = F(1) if v > F(1) else v

    def setp(self, i, p):
        p = F(p)
        if self.kind == 1:
            if self.prob[i] < p:
                self.prob[i] = p
                self.hit[i] = F(p * self.pas[i])
        elif self.prob[i] < p and p <= F(1):
            self.prob[i] = p

    def inmap(self, x, y, tol=0.0):
        return x > tol and x < self.sx - tol and y > tol and y < self.sy - tol

    def cell_update(self, x, y, typ):
        if not self.inmap(x, y, self.hk + 1):
            return
        i = y * self.row + x
        if typ == 0:
            if self.uidx[i] < self.cf:
                self.free(i)
                self.uidx[i] = self.cf
            self.points.append(i)
        elif typ == 1:
            if self.uidx[i] < self.co:
                if self.uidx[i] == self.cf:
                    self.unfree(i)
                self.occ(i)
                self.uidx[i] = self.co
            self.points.append(i)
        else:
            if self.uidx[i] < self.co:
                if not self.just:
                    if self.uidx[i] == self.cf:
                        self.unfree(i)
                    self.occ(i)
                    self.uidx[i] = self.co
                else:
                    self.setp(i, 1.0)
                ks = 2 * self.hk + 1
                for j in range(-self.hk, self.hk + 1):
                    for ii in range(-self.hk, self.hk + 1):
                        k = (ii + self.hk) + ks * (j + self.hk)
                        c = (y + j) * self.row + (x + ii)
                        self.setp(c, F(self.kern[k] * self.offs))
                        self.points.append(c)

    def extend(self):
        tmin = [FLT_MAX, FLT_MAX]
        tmax = [FLT_MIN, FLT_MIN]

        def add(p):
            for a in range(2):
                if p[a] < tmin[a]:
                    tmin[a] = p[a]
                if p[a] > tmax[a]:
                    tmax[a] = p[a]

        add(self.bmin), add(self.bmax)
        add([0.0, 0.0]), add([float(self.sx), float(self.sy)])
        size = [int(math.ceil(tmax[a]) - math.floor(tmin[a])) for a in range(2)]
        lo, hi = list(tmin), list(tmax)
        mapmax = [float(self.sx), float(self.sy)]
        for a in range(2):
            if self.bmin[a] <= 0.0:
                lo[a] -= float(size[a]) * self.ext
            if self.bmax[a] >= mapmax[a]:
                hi[a] += float(size[a]) * self.ext
        add(lo), add(hi)
        fl = [math.floor(tmin[0]), math.floor(tmin[1])]
        self.ox -= fl[0] / self.s
        self.oy -= fl[1] / self.s
        gx, gy = -int(fl[0]), -int(fl[1])
        nsx = int(math.ceil(tmax[0]) - math.floor(tmin[0]))
        nsy = int(math.ceil(tmax[1]) - math.floor(tmin[1]))
        n = nsx * nsy
        prob = [F(0.5)] * n
        prob[0] = self.dflt
        pas, hit, uidx = [F(0)] * n, [F(0)] * n, [-1] * n
        for r in range(self.sy):
            for x in range(self.row):
                d = (gy + r) * nsx + gx + x
                s = r * self.row + x
                prob[d], pas[d], hit[d], uidx[d] = self.prob[s], self.pas[s], self.hit[s], self.uidx[s]
        self.prob, self.pas, self.hit, self.uidx = prob, pas, hit, uidx
        self.row, self.sx, self.sy = nsx, nsx, nsy
        self.bmin = [self.bmin[0] - tmin[0], self.bmin[1] - tmin[1]]
        self.bmax = [self.bmax[0] - tmin[0], self.bmax[1] - tmin[1]]

    def update(self, pts, pose, use_blur=False, origin=(0.0, 0.0)):
        if not self.blur_ok:
            use_blur = False
        self.cf, self.co = self.cur + 1, self.cur + 2
        s = self.s
        px, py, th = s * pose[0] + s * self.ox, s * pose[1] + s * self.oy, pose[2]
        c, sn = sincos(th)
        tp = [((c * x + (-sn) * y) + px, (sn * x + c * y) + py) for x, y in pts]
        if self.auto and tp:
            bmin = [FLT_MAX, FLT_MAX]
            bmax = [FLT_MIN, FLT_MIN]
            for p in tp:
                for a in range(2):
                    if p[a] < bmin[a]:
                        bmin[a] = p[a]
                    if p[a] > bmax[a]:
                        bmax[a] = p[a]
            if use_blur:
                bmin = [v - float(self.hk) for v in bmin]
                bmax = [v + float(self.hk) for v in bmax]

            def inb(p):
                return (p[0] > self.bmin[0] and p[0] < self.bmax[0] and p[1] > self.bmin[1]
                        and p[1] < self.bmax[1])

            if not (inb(bmin) and inb(bmax)):
                for p in (bmin, bmax):
                    for a in range(2):
                        if p[a] < self.bmin[a]:
                            self.bmin[a] = p[a]
                        if p[a] > self.bmax[a]:
                            self.bmax[a] = p[a]
                if not self.inmap(*self.bmin) or not self.inmap(*self.bmax):
                    self.extend()
                    self.cur += 3
                    return False
        sxo, syo = (c * origin[0] + (-sn) * origin[1]) + px, (sn * origin[0] + c * origin[1]) + py
        x0, y0 = int(sxo + 0.5), int(syo + 0.5)
        for ex, ey in tp:
            x1, y1 = int(ex + 0.5), int(ey + 0.5)
            if (x0, y0) != (x1, y1):
                if not self.just:
                    for x, y in bresenham(x0, y0, x1, y1):
                        self.cell_update(x, y, 0)
                self.cell_update(x1, y1, 2 if use_blur else 1)
        self.mui += 1
        self.cur += 3
        return True

    def init_vec(self, scans, poses, use_blur=False, speedup=False):
        if speedup:
            for i in self.points:
                self._reset(i)
        else:
            for i in range(len(self.prob)):
                self._reset(i)
        self.cur, self.co, self.cf = 0, -1, -1
        self.points = []
        for pts, pose in zip(scans, poses):
            tries = 5
            while not self.update(pts, pose, use_blur) and tries:
                tries -= 1
        if not self.auto:
            self.bmin = [0.0, 0.0]
            self.bmax = [float(self.sx + 1), float(self.sy + 1)]

    def _reset(self, i):
        self.prob[i], self.pas[i], self.hit[i], self.uidx[i] = self.dflt, F(0), F(0), -1

    def arrays(self):
        sh = (self.sy, self.sx)
        return (np.array(self.prob, dtype=np.float32).reshape(sh), np.array(self.pas, dtype=np.float32).reshape(sh),
                np.array(self.hit, dtype=np.float32).reshape(sh), np.array(self.uidx, dtype=np.int32).reshape(sh))

    def touched(self):
        f = np.zeros(len(self.prob), dtype=np.uint8)
        for i in self.points:
            f[i] = 1
        return f

    def penalty(self, pts, pose, check_point_num, tol, gain, use_blur=False, origin=(0.0, 0.0)):
        """MapFeedbackResponsePenalty (occu_grid_map.h:331-392)."""
        if tol < 0 or check_point_num <= 0 or gain <= 0.0 or gain >= 1.0:
            return 1.0
        s = self.s
        px, py, th = s * pose[0] + s * self.ox, s * pose[1] + s * self.oy, pose[2]
        if not self.inmap(px, py):
            return 0.0
        c, sn = sincos(th)
        x0 = int(((c * origin[0] + (-sn) * origin[1]) + px) + 0.5)
        y0 = int(((sn * origin[0] + c * origin[1]) + py) + 0.5)
        n = len(pts)
        step = 1 if n < 2 * check_point_num else n // (check_point_num - 1)
        pen = 0.0
        for i in range(0, n, step):
            x, y = pts[i]
            x1 = int(((c * x + (-sn) * y) + px) + 0.5)
            y1 = int(((sn * x + c * y) + py) + 0.5)
            if (x0, y0) == (x1, y1) or not self.inmap(x1, y1):
                continue
            res = 0.0
            for cx, cy in bresenham(x0, y0, x1, y1):
                ps = 0.0
                occ = False
                if 0 <= cx < self.sx and 0 <= cy < self.sy:
                    i2 = cy * self.row + cx
                    if use_blur:
                        occ = float(self.prob[i2]) > self.offs
                    elif self.kind == 1:
                        occ = self.pas[i2] >= self.mp and not (self.prob[i2] < self.thr)
                    else:
                        occ = self.prob[i2] > F(0.5)
                if occ and math.sqrt(float(x1 - cx) ** 2 + float(y1 - cy) ** 2) > tol:
                    ps += 1.0
                if res < 1.0:
                    res += ps
            pen += res
        pen *= gain
        return max(1.0 + 2 * gain - pen, 0.1)
