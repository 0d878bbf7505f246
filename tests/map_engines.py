"""Uniform adapters over the three map implementations used by the map
tests: the oracle (pyoracle.GridMap), the independent Python restatement
(map_pyref.PyMap) and the device maps (roborts_csm.gridmap.OccuGridMap)."""
from __future__ import annotations

import numpy as np


class OracleEngine:
    def __init__(self, kind, res, size, off, dev, default):
        import pyoracle as O
        self.m = O.GridMap(kind, res, size, off, dev, default)

    def set_options(self, auto, just, offs, ext):
        self.m.set_options(auto, just, offs, ext)

    def set_cell_params(self, ff, fo, thr, mp):
        self.m.set_cell_params(ff, fo, thr, mp)

    def update(self, pts, pose, blur):
        return self.m.update_by_range(pts, pose, use_blur=blur)

    def init(self, scans, poses, blur, speedup):
        self.m.init_with_range_vec(scans, poses, use_blur=blur, speedup=speedup)

    def set_offset(self, o):
        self.m.set_map_offset(*o)

    def state(self):
        return self.m.info()

    def penalty(self, pts, pose, n, tol, gain, blur):
        return self.m.feedback_penalty(pts, pose, n, tol, gain, use_blur=blur)

    def arrays(self):
        p, ps, h, u = self.m.cells()
        return p, ps, h, u, self.m.touched().reshape(p.shape)


class PyrefEngine:
    def __init__(self, kind, res, size, off, dev, default):
        from map_pyref import PyMap
        self.m = PyMap(kind, res, size, off, dev, default)

    def set_options(self, auto, just, offs, ext):
        self.m.auto, self.m.just, self.m.offs = auto, just, offs
        if ext > 0:
            self.m.ext = ext

    def set_cell_params(self, ff, fo, thr, mp):
        m = self.m
        m.ff, m.fo = np.float32(ff), np.float32(fo)
        if m.kind == 1:
            m.thr, m.mp = np.float32(thr), np.float32(mp)

    def update(self, pts, pose, blur):
        return self.m.update([tuple(p) for p in np.asarray(pts)], pose, blur)

    def init(self, scans, poses, blur, speedup):
        self.m.init_vec([[tuple(p) for p in np.asarray(s)] for s in scans], poses, blur, speedup)

    def set_offset(self, o):
        self.m.ox, self.m.oy = o

    def state(self):
        m = self.m
        return {"size_x": m.sx, "size_y": m.sy, "map_update_index": m.mui, "cur_update_index": m.cur,
                "offset": (m.ox, m.oy), "bound": (m.bmin[0], m.bmin[1], m.bmax[0], m.bmax[1])}

    def penalty(self, pts, pose, n, tol, gain, blur):
        return self.m.penalty([tuple(p) for p in np.asarray(pts)], pose, n, tol, gain, blur)

    def arrays(self):
        p, ps, h, u = self.m.arrays()
        return p, ps, h, u, self.m.touched().reshape(p.shape)


class DeviceEngine:
    def __init__(self, kind, res, size, off, dev, default):
        from roborts_csm.gridmap import OccuGridMap
        self.m = OccuGridMap(res, size, off, dev, default, kind=kind)

    def set_options(self, auto, just, offs, ext):
        self.m.set_options(auto, just, offs, ext)

    def set_cell_params(self, ff, fo, thr, mp):
        self.m.set_cell_params(ff, fo, thr, mp)

    def update(self, pts, pose, blur):
        return self.m.UpdateMapByRange(pts, pose, use_blur=blur)

    def init(self, scans, poses, blur, speedup):
        self.m.InitMapWithRangeVec(scans, poses, use_blur=blur, use_reset_speedup=speedup)

    def set_offset(self, o):
        self.m.set_map_offset(o)

    def state(self):
        s = self.m.state()
        return {"size_x": s.size_x, "size_y": s.size_y, "map_update_index": s.map_update_index,
                "cur_update_index": s.cur_update_index, "offset": (s.offset_x, s.offset_y),
                "bound": (s.bound_min_x, s.bound_min_y, s.bound_max_x, s.bound_max_y)}

    def penalty(self, pts, pose, n, tol, gain, blur):
        return self.m.MapFeedbackResponsePenalty(pts, pose, n, tol, gain, use_blur=blur)

    def arrays(self):
        return self.m.cells()


def same_state(a, b):
    """Bit-identical cells (NaN-aware), update indices, touched set and geometry."""
    sa, sb = a.state(), b.state()
    for k in ("size_x", "size_y", "map_update_index", "cur_update_index"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    assert tuple(sa["offset"]) == tuple(sb["offset"]), (sa["offset"], sb["offset"])
    assert tuple(sa["bound"]) == tuple(sb["bound"]), (sa["bound"], sb["bound"])
    for name, x, y in zip(("prob", "pass", "hit", "update_index", "touched"), a.arrays(), b.arrays()):
        assert x.shape == y.shape, name
        xv, yv = x.view(np.uint32) if x.dtype == np.float32 else x, y.view(np.uint32) if y.dtype == np.float32 else y
        bad = np.flatnonzero(xv.ravel() != yv.ravel())
        assert bad.size == 0, f"{name}: {bad.size} cells differ, first {bad[:5]}: {x.ravel()[bad[:5]]} vs {y.ravel()[bad[:5]]}"
