"""roborts_csm — MI355X-native correlative scan matcher for RoboRTS-Edu-SLAM.

Python mirror of the reference's scan-matching interface, bound to the C-ABI
of libroborts_csm.so (include/csm.h). Names, argument meaning and error
behaviour follow the reference:

  ScanMatchMap                 ~ ScanMatchMap = OccuGridMap<ProbabilityCell> (map/slam_map.h:32-34)
  RangeDataContainer2d         ~ RangeDataContainer<double> (slam/sensor_data_manager.h:87-300)
  BasedCorrelationScanMatch    ~ correlate_scan_matcher.h:766-1036 (ScanMatch :784-875)
  ScanMatchers                 ~ scan_match/scan_matchers.h:160-416 (ScanMatch :179-289)

Everything numeric runs in the shared library on the GPU; this module only
moves arrays. Importing it fails loudly when the library is missing.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

from . import _abi
from ._abi import COARSE, FAST, FINE, SUPER, CsmBest, CsmMapInfo, CsmParam
from .params import (
    CONFIG1_PARAM, FAST_PARAM, IN_CLASS_LEVELS, PARAM_CONFIG_LEVELS, PARAM_CONFIG_OPTIMIZE, SIM_YAML_LEVELS,
    SIM_YAML_OPTIMIZE, CorrelationScanMatchParam, OptimizeScanMatchParam, headline_levels,
)

_lib = _abi.load_library()

kMapUnknownCellProb = np.float32(0.3)  # slam/slam_processor.h:264


class CsmError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"csm status {status}: {msg}")
        self.status = status


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _i64ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def _as_param(p) -> CsmParam:
    if isinstance(p, CsmParam):
        return p
    return p.to_c()


# ---------------------------------------------------------------------------
# Data containers (reference data formats either side of the boundary)
# ---------------------------------------------------------------------------

@dataclass
class ScanMatchMap:
    """Probability grid + GridMapBase geometry (map/grid_map_base.h:47-71).

    ``cells`` is either a packed float32 [size_y, size_x] array or the
    reference's AoS ProbabilityCell layout as a structured array with fields
    (prob_value_ f4, update_index_ i4) (map/grid_map_cell.h:301-328).
    """

    cells: np.ndarray
    resolution: float
    offset: tuple = (0.0, 0.0)
    update_index: int = 0
    version: int = 0

    @property
    def size_x(self) -> int:
        return int(self.cells.shape[1])

    @property
    def size_y(self) -> int:
        return int(self.cells.shape[0])

    def IsMapInit(self) -> bool:  # grid_map_base.h:373-378
        return self.update_index >= 0

    def GetCellLength(self) -> float:  # grid_map_base.h:307-309
        return 1 / (1.0 / self.resolution)

    def info(self) -> CsmMapInfo:
        return CsmMapInfo(float(self.resolution), float(self.offset[0]), float(self.offset[1]),
                          self.size_x, self.size_y, int(self.update_index), 0)

    def GetMapCoordsPose(self, pose_world) -> np.ndarray:  # grid_map_base.h:89-93
        s = 1.0 / self.resolution
        return np.array([s * pose_world[0] + s * self.offset[0],
                         s * pose_world[1] + s * self.offset[1], pose_world[2]])

    def GetWorldCoordsPose(self, pose_map) -> np.ndarray:  # grid_map_base.h:83-87
        s = 1.0 / self.resolution
        a = s * (1.0 / (s * s - 0.0 * 0.0))
        return np.array([a * pose_map[0] + -(a * (s * self.offset[0])),
                         a * pose_map[1] + -(a * (s * self.offset[1])), pose_map[2]])


@dataclass
class RangeDataContainer2d:
    """Scan endpoints in the sensor frame (slam/sensor_data_manager.h:87-300)."""

    points: np.ndarray = field(default_factory=lambda: np.zeros((0, 2)))
    sensor_pose: np.ndarray = field(default_factory=lambda: np.zeros(3))
    scale_factor: float = 1.0

    def CreateFrom(self, other: "RangeDataContainer2d", factor: float) -> "RangeDataContainer2d":
        """Copy and scale every point by ``factor`` (sensor_data_manager.h:99-115)."""
        self.scale_factor = factor
        self.sensor_pose = np.array(other.sensor_pose, dtype=np.float64)
        self.points = np.ascontiguousarray(other.points, dtype=np.float64) * factor
        return self

    def GetSize(self) -> int:
        return int(self.points.shape[0])

    def GetDataPoint(self, i: int) -> np.ndarray:
        return self.points[i]


def cell_points(points_m: np.ndarray, resolution: float) -> np.ndarray:
    """Metres -> map cells as CreateFrom(range, 1 / resolution) does."""
    return np.ascontiguousarray(points_m, dtype=np.float64) * (1 / resolution)


# ---------------------------------------------------------------------------
# Context over the C-ABI
# ---------------------------------------------------------------------------

class Context:
    """One csm_ctx: a device, a HIP stream, a resident grid."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        st = _lib.csm_create(int(device), C.byref(h))
        if st != _abi.CSM_OK:
            raise CsmError(st, f"csm_create(device={device}) failed (no usable HIP device?)")
        self._h = h
        self.device = device
        self._grid_ref = None

    @classmethod
    def borrow(cls, handle, owner) -> "Context":
        """A view of a context another object owns (csm_frontend_matcher):
        close() does not destroy it; `owner` is kept alive meanwhile."""
        c = cls.__new__(cls)
        c._h = handle
        c.device = None
        c._grid_ref = None
        c._owner = owner
        return c

    def close(self):
        if getattr(self, "_owner", None) is not None:  # borrowed
            self._h = None
            self._owner = None
            return
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.csm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st: int):
        if st != _abi.CSM_OK:
            raise CsmError(st, _lib.csm_last_error(self._h).decode())

    def sincos_device(self, x):
        """(sin x, cos x) computed on the GPU as the 3-level driver's angle rows
        are (csm_sincos_device: glibc's sincos restated, bit-equal to the host's)."""
        a = np.ascontiguousarray(x, dtype=np.float64).ravel()
        s = np.empty_like(a)
        c = np.empty_like(a)
        self._check(_lib.csm_sincos_device(self._h, a.ctypes.data_as(_abi._dp), a.size,
                                           s.ctypes.data_as(_abi._dp), c.ctypes.data_as(_abi._dp)))
        return s, c

    def set_outside_value(self, v: float):
        self._check(_lib.csm_set_outside_value(self._h, C.c_float(v)))

    def set_grid(self, m: ScanMatchMap, force: bool = False):
        cells = m.cells
        if cells.dtype == np.float32:
            cells = np.ascontiguousarray(cells)
            stride = 4
        elif cells.dtype.names and "prob_value_" in cells.dtype.names:
            cells = np.ascontiguousarray(cells)
            stride = cells.dtype.itemsize
        else:
            raise TypeError("grid cells must be float32 or a ProbabilityCell structured array")
        self._keep(cells)
        info = m.info()
        self._check(_lib.csm_set_grid(self._h, cells.ctypes.data_as(C.c_void_p), stride,
                                      C.byref(info), -1 if force else int(m.version)))

    def _keep(self, cells):
        """Keep host grids alive while the library may key resident copies on
        their address (up to four maps stay resident)."""
        refs = self.__dict__.setdefault("_grid_refs", {})
        refs.pop(cells.ctypes.data, None)
        refs[cells.ctypes.data] = cells
        while len(refs) > 8:
            refs.pop(next(iter(refs)))

    @staticmethod
    def _cells_of(m: ScanMatchMap):
        cells = m.cells
        if cells.dtype == np.float32:
            stride = 4
        elif cells.dtype.names and "prob_value_" in cells.dtype.names:
            stride = cells.dtype.itemsize
        else:
            raise TypeError("grid cells must be float32 or a ProbabilityCell structured array")
        if not cells.flags.c_contiguous:
            raise ValueError("incremental refresh needs the map's own contiguous cell array")
        return cells, stride

    def update_grid_cells(self, m: ScanMatchMap, cell_indices):
        """csm_update_grid_cells: re-read the listed cells (y*size_x + x) of a
        resident map after an in-place update; m.version is the new key."""
        cells, stride = self._cells_of(m)
        self._keep(cells)
        idx = np.ascontiguousarray(cell_indices, dtype=np.int32).ravel()
        info = m.info()
        self._check(_lib.csm_update_grid_cells(self._h, cells.ctypes.data_as(C.c_void_p), stride, C.byref(info),
                                               int(m.version), idx.ctypes.data_as(_abi._i32p), idx.size))

    def update_grid_rows(self, m: ScanMatchMap, row_begin: int, row_end: int):
        """csm_update_grid_rows: re-read rows [row_begin, row_end)."""
        cells, stride = self._cells_of(m)
        self._keep(cells)
        info = m.info()
        self._check(_lib.csm_update_grid_rows(self._h, cells.ctypes.data_as(C.c_void_p), stride, C.byref(info),
                                              int(m.version), int(row_begin), int(row_end)))

    def set_grid_device(self, dev_ptr: int, m: ScanMatchMap):
        info = m.info()
        self._check(_lib.csm_set_grid_device(self._h, C.c_void_p(dev_ptr), C.byref(info)))

    # -- reference entry points -------------------------------------------
    def scan_match(self, points_cells: np.ndarray, param, pose: np.ndarray, cov: np.ndarray,
                   return_argmax: bool = False):
        """BasedCorrelationScanMatch::ScanMatch; pose/cov updated in place."""
        pts = np.ascontiguousarray(points_cells, dtype=np.float64).reshape(-1, 2)
        assert pose.dtype == np.float64 and pose.flags.c_contiguous and pose.size == 3
        assert cov.dtype == np.float64 and cov.flags.c_contiguous and cov.size == 9
        p = _as_param(param)
        resp = C.c_double(0.0)
        am = C.c_int64(-1)
        self._loaded = None  # host points replace the loaded set (include/csm.h)
        self._check(_lib.csm_scan_match(self._h, _dptr(pts), pts.shape[0], C.byref(p), _dptr(pose),
                                        _dptr(cov), C.byref(resp), C.byref(am)))
        return (resp.value, am.value) if return_argmax else resp.value

    def scan_matchers(self, points_cells, levels: Sequence, pose, cov, use_fine: bool = True) -> float:
        pts = np.ascontiguousarray(points_cells, dtype=np.float64).reshape(-1, 2)
        lv = (CsmParam * 3)(*[_as_param(l) for l in levels])
        sc = C.c_double(0.0)
        # csm_scan_matchers loads, dropping queued batches: their arrays stay
        # referenced until the call (which waits for their uploads) returns
        queued = self.__dict__.get("_queued")
        self._loaded = (pts, np.array([0, pts.shape[0]], dtype=np.int64))  # it is the loaded set now
        try:
            self._check(_lib.csm_scan_matchers(self._h, _dptr(pts), pts.shape[0], lv, 1 if use_fine else 0,
                                               _dptr(pose), _dptr(cov), C.byref(sc)))
        finally:
            if queued is not None and self.__dict__.get("_queued") is queued:
                self.__dict__.pop("_queued", None)
        return sc.value

    def scan_match_batch(self, points: np.ndarray, offsets: np.ndarray, param, poses, covs):
        """Returns (responses, argmax_flat) for n independent scans."""
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 2)
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        n = off.size - 1
        assert poses.dtype == np.float64 and poses.flags.c_contiguous and poses.size == 3 * n
        assert covs.dtype == np.float64 and covs.flags.c_contiguous and covs.size == 9 * n
        resp = np.zeros(n)
        am = np.full(n, -1, dtype=np.int64)
        p = _as_param(param)
        self._loaded = None  # host points replace the loaded set (include/csm.h)
        self._check(_lib.csm_scan_match_batch(self._h, n, _dptr(pts), _i64ptr(off), C.byref(p),
                                              _dptr(poses), _dptr(covs), _dptr(resp), _i64ptr(am)))
        return resp, am

    def scan_matchers_batch(self, points, offsets, levels, poses, covs, use_fine: bool = True):
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 2)
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        n = off.size - 1
        assert poses.dtype == np.float64 and poses.flags.c_contiguous and poses.size == 3 * n
        assert covs.dtype == np.float64 and covs.flags.c_contiguous and covs.size == 9 * n
        scores = np.zeros(n)
        lv = (CsmParam * 3)(*[_as_param(l) for l in levels])
        queued = self.__dict__.get("_queued")  # a synchronous load drops queued batches (after the call)
        self._loaded = (pts, off)  # it is the loaded set now
        try:
            self._check(_lib.csm_scan_matchers_batch(self._h, n, _dptr(pts), _i64ptr(off), lv,
                                                     1 if use_fine else 0, _dptr(poses), _dptr(covs),
                                                     _dptr(scores)))
        finally:
            if queued is not None and self.__dict__.get("_queued") is queued:
                self.__dict__.pop("_queued", None)
        return scores

    def load_scans(self, points, offsets):
        """Make a batch of scans device-resident (csm_load_scans)."""
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 2)
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        self._loaded = (pts, off)
        queued = self.__dict__.get("_queued")  # the library drops queued batches too (after the call)
        try:
            self._check(_lib.csm_load_scans(self._h, off.size - 1, _dptr(pts), _i64ptr(off)))
        finally:
            if queued is not None and self.__dict__.get("_queued") is queued:
                self.__dict__.pop("_queued", None)

    def load_scans_async(self, points, offsets):
        """Queue a batch (csm_load_scans_async): its upload runs beside the
        current match; the next scan_matchers_loaded / scan_matchers_submit
        takes it (load_scans, scan_matchers and scan_matchers_batch drop it).
        `points` should be pinned (a PinnedArray's array) and must not change
        until then; the arrays are kept referenced here meanwhile."""
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 2)
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        q = self.__dict__.setdefault("_queued", [])
        self._check(_lib.csm_load_scans_async(self._h, off.size - 1, _dptr(pts), _i64ptr(off)))
        q.append((pts, off))

    def _take_loaded(self) -> int:
        """The scan count of the batch the next loaded / submitted match runs."""
        q = self.__dict__.get("_queued")
        if q:  # the library takes the oldest queued batch
            self._loaded = q.pop(0)
        if self.__dict__.get("_loaded") is None:
            raise CsmError(_abi.CSM_ERR_INVALID_ARG, "no scans loaded (csm_load_scans)")
        return self._loaded[1].size - 1

    def scan_matchers_loaded(self, levels, poses, covs, use_fine: bool = True):
        n = self._take_loaded()
        assert poses.dtype == np.float64 and poses.flags.c_contiguous and poses.size == 3 * n
        assert covs.dtype == np.float64 and covs.flags.c_contiguous and covs.size == 9 * n
        scores = np.zeros(n)
        lv = (CsmParam * 3)(*[_as_param(l) for l in levels])
        self._check(_lib.csm_scan_matchers_loaded(self._h, lv, 1 if use_fine else 0, _dptr(poses),
                                                  _dptr(covs), _dptr(scores)))
        return scores

    def scan_matchers_submit(self, levels, poses, covs, scores, use_fine: bool = True):
        """csm_scan_matchers_submit: scan_matchers_loaded with the batch's last
        level left pending; poses / covs / scores (float64, caller-owned) are
        final after the next submit, scan_matchers_wait() or any other call,
        and must stay alive until then (they are kept referenced here). The
        oldest queued batch (load_scans_async) is taken first, as by
        scan_matchers_loaded, without completing the pending one."""
        n = self._take_loaded()
        for a, k in ((poses, 3), (covs, 9), (scores, 1)):
            assert a.dtype == np.float64 and a.flags.c_contiguous and a.size == k * n
        lv = (CsmParam * 3)(*[_as_param(l) for l in levels])
        keep = self.__dict__.setdefault("_submitted", [])
        keep.append((poses, covs, scores))
        del keep[:-2]  # the two batches the library may still write
        self._check(_lib.csm_scan_matchers_submit(self._h, lv, 1 if use_fine else 0, _dptr(poses), _dptr(covs),
                                                  _dptr(scores)))

    def scan_matchers_wait(self):
        self._check(_lib.csm_scan_matchers_wait(self._h))

    def optimize_scan_match(self, points_cells, param, pose: np.ndarray) -> float:
        """BasedOptimizeScanMatch::ScanMatch on the current grid; pose updated in place."""
        pts = np.ascontiguousarray(points_cells, dtype=np.float64).reshape(-1, 2)
        assert pose.dtype == np.float64 and pose.flags.c_contiguous and pose.size == 3
        p = param if isinstance(param, _abi.CsmOptimizeParam) else param.to_c()
        cost = C.c_double(0.0)
        self._check(_lib.csm_optimize_scan_match(self._h, _dptr(pts), pts.shape[0], C.byref(p), _dptr(pose),
                                                 C.byref(cost)))
        return cost.value

    def optimize_scan_match_batch(self, points, offsets, param, poses):
        """Returns (costs, iterations) for n independent scans; poses updated in place."""
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 2)
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        n = off.size - 1
        assert poses.dtype == np.float64 and poses.flags.c_contiguous and poses.size == 3 * n
        p = param if isinstance(param, _abi.CsmOptimizeParam) else param.to_c()
        costs = np.zeros(n)
        iters = np.zeros(n, dtype=np.int32)
        self._check(_lib.csm_optimize_scan_match_batch(self._h, n, _dptr(pts), _i64ptr(off), C.byref(p),
                                                       _dptr(poses), _dptr(costs),
                                                       iters.ctypes.data_as(C.POINTER(C.c_int32))))
        return costs, iters

    def optimize_update_cost(self, points_cells, est_map):
        """One device UpdateCost at a map-cell pose -> (cost, H 3x3, b) (test hook)."""
        pts = np.ascontiguousarray(points_cells, dtype=np.float64).reshape(-1, 2)
        est = np.ascontiguousarray(est_map, dtype=np.float64)
        cost, H, b = C.c_double(0.0), np.zeros(9), np.zeros(3)
        self._check(_lib.csm_optimize_update_cost(self._h, _dptr(pts), pts.shape[0], _dptr(est), C.byref(cost),
                                                  _dptr(H), _dptr(b)))
        return cost.value, H.reshape(3, 3), b

    def sort_order(self, keys) -> np.ndarray:
        """Device emulation of std::sort(greater) on keys (test hook)."""
        k = np.ascontiguousarray(keys, dtype=np.float64)
        out = np.empty(k.size, dtype=np.int64)
        self._check(_lib.csm_sort_order(self._h, _dptr(k), k.size, _i64ptr(out)))
        return out

    def host_plan(self) -> dict:
        """csm_get_host_plan: the CPUs and thread count of this context's pool."""
        p = _abi.CsmHostPlan()
        self._check(_lib.csm_get_host_plan(self._h, C.byref(p)))
        return p.as_dict()

    def set_profiling(self, on=True):
        """True/1: time every scoring launch and finish; 2: the 3-level
        drivers' first-level scoring kernels only (csm.h csm_set_profiling);
        False/0: off."""
        self._check(_lib.csm_set_profiling(self._h, int(on) if on in (0, 1, 2) else (1 if on else 0)))

    def kernel_stats(self) -> list[dict]:
        cnt = C.c_int32(0)
        self._check(_lib.csm_kernel_stats(self._h, None, 0, C.byref(cnt)))
        arr = (_abi.CsmKernelStat * max(cnt.value, 1))()
        self._check(_lib.csm_kernel_stats(self._h, arr, cnt.value, C.byref(cnt)))
        return [dict(name=a.name.decode(), launches=a.launches, total_ms=a.total_ms,
                     algorithmic_bytes=a.algorithmic_bytes, scorings=a.scorings) for a in arr[:cnt.value]]

    def score_window(self, points_cells, param, center_map) -> np.ndarray:
        pts = np.ascontiguousarray(points_cells, dtype=np.float64).reshape(-1, 2)
        p = _as_param(param)
        na, ns = window_dims(p)
        out = np.empty(na * ns * ns)
        ctr = np.ascontiguousarray(center_map, dtype=np.float64)
        self._check(_lib.csm_score_window(self._h, _dptr(pts), pts.shape[0], C.byref(p), _dptr(ctr),
                                          _dptr(out), out.size))
        return out

    def best_window(self, points_cells, param, center_map) -> CsmBest:
        pts = np.ascontiguousarray(points_cells, dtype=np.float64).reshape(-1, 2)
        p = _as_param(param)
        ctr = np.ascontiguousarray(center_map, dtype=np.float64)
        b = CsmBest()
        self._check(_lib.csm_best_window(self._h, _dptr(pts), pts.shape[0], C.byref(p), _dptr(ctr),
                                         C.byref(b)))
        return b

    def set_grid_stack(self, grids: np.ndarray, resolution: float, version: int = -1) -> None:
        """Resident stack of same-size fp32 grids (loop-closure submaps)."""
        g = np.ascontiguousarray(grids, dtype=np.float32)
        assert g.ndim == 3
        self._stack = g  # the cache key is the host pointer: keep it alive
        info = CsmMapInfo(float(resolution), 0.0, 0.0, g.shape[2], g.shape[1], 0, 0)
        self._check(_lib.csm_set_grid_stack(self._h, g.ctypes.data_as(C.c_void_p), g.shape[0], C.byref(info),
                                            int(version)))

    def best_windows(self, points_cells, param, grid_index, centers_map):
        """Argmax of one scan over many windows -> (scores, flat, x, y, angle) arrays."""
        pts = np.ascontiguousarray(points_cells, dtype=np.float64).reshape(-1, 2)
        p = _as_param(param)
        gi = np.ascontiguousarray(grid_index, dtype=np.int32)
        ctr = np.ascontiguousarray(centers_map, dtype=np.float64).reshape(-1, 3)
        assert gi.size == ctr.shape[0]
        out = (CsmBest * max(1, gi.size))()
        self._check(_lib.csm_best_windows(self._h, _dptr(pts), pts.shape[0], C.byref(p), gi.size,
                                          gi.ctypes.data_as(C.POINTER(C.c_int32)), _dptr(ctr), out))
        n = gi.size
        return (np.array([out[i].score for i in range(n)]), np.array([out[i].flat_index for i in range(n)]),
                np.array([out[i].x for i in range(n)]), np.array([out[i].y for i in range(n)]),
                np.array([out[i].angle for i in range(n)]))


    def search_windows(self, points_cells, param, grid_index, centers_map, max_depth: int = -1,
                       probe_min_nodes: int = 0, node_capacity: int = 0, top_kernel: int = 0):
        """Best candidate of one scan over many windows by the admissible
        multi-resolution search (csm_search_windows) -> (CsmBest, window, stats
        dict). Same answer as reducing best_windows: max score, lowest
        (window, flat index)."""
        pts = np.ascontiguousarray(points_cells, dtype=np.float64).reshape(-1, 2)
        p = _as_param(param)
        gi = np.ascontiguousarray(grid_index, dtype=np.int32)
        ctr = np.ascontiguousarray(centers_map, dtype=np.float64).reshape(-1, 3)
        assert gi.size == ctr.shape[0]
        opt = _abi.CsmSearchOptions(int(max_depth), int(probe_min_nodes), int(node_capacity), int(top_kernel), 0)
        b = CsmBest()
        w = C.c_int32(-1)
        st = _abi.CsmSearchStats()
        self._check(_lib.csm_search_windows(self._h, _dptr(pts), pts.shape[0], C.byref(p), gi.size,
                                            gi.ctypes.data_as(C.POINTER(C.c_int32)), _dptr(ctr), C.byref(opt),
                                            C.byref(b), C.byref(w), C.byref(st)))
        stats = dict(depth=st.depth, exhaustive=bool(st.exhaustive), candidates=st.candidates,
                     nodes=list(st.nodes), probe_leaves=st.probe_leaves, beam_reads=st.beam_reads,
                     build_ms=st.build_ms, syncs=st.syncs, top_box=bool(st.top_box))
        return b, int(w.value), stats


class _PinnedBlock:
    """One csm_host_alloc allocation, freed when the last array over it dies."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        if _lib.csm_host_alloc(max(1, nbytes), C.byref(p)) != 0:
            raise MemoryError("csm_host_alloc failed")
        self.p = p

    def __del__(self):
        try:
            if self.p is not None and self.p.value:
                _lib.csm_host_free(self.p)
            self.p = None
        except Exception:
            pass


class PinnedArray:
    """A numpy array over pinned host memory (csm_host_alloc), for
    load_scans_async inputs. The allocation belongs to the array's buffer
    (``array.base``), so it lives as long as any view of it does: close()
    only drops this object's reference."""

    def __init__(self, shape, dtype=np.float64):
        self.dtype = np.dtype(dtype)
        n = int(np.prod(shape))
        nbytes = max(1, n) * self.dtype.itemsize
        block = _PinnedBlock(nbytes)
        buf = (C.c_char * nbytes).from_address(block.p.value)
        buf._block = block  # the numpy array's base keeps the allocation alive
        self.array = np.frombuffer(buf, dtype=self.dtype, count=n).reshape(shape)

    def close(self):
        self.array = None


def host_plan(local_rank: int, local_world: int, numa_of_rank=None, quota_cpus: int = 0) -> dict:
    """csm_host_plan_compute (no GPU needed): the pool a context of local rank
    `local_rank` of `local_world` would get. numa_of_rank: each local rank's
    GPU NUMA node (None: unknown); quota_cpus: 0 reads the cgroup, -1 none."""
    p = _abi.CsmHostPlan()
    arr = None
    if numa_of_rank is not None:
        arr = np.ascontiguousarray(numa_of_rank, dtype=np.int32)
        assert arr.size == local_world
    st = _lib.csm_host_plan_compute(int(local_rank), int(local_world),
                                    None if arr is None else arr.ctypes.data_as(_abi._i32p), int(quota_cpus),
                                    C.byref(p))
    if st != _abi.CSM_OK:
        raise CsmError(st, "csm_host_plan_compute: invalid rank / world")
    return p.as_dict()


def build_digest() -> str:
    """The source digest the loaded library was compiled from (csm_build_digest;
    tools/source_digest.py computes the tree's)."""
    return _lib.csm_build_digest().decode()


def window_dims(param) -> tuple[int, int]:
    p = _as_param(param)
    na, ns = C.c_int32(), C.c_int32()
    st = _lib.csm_window_dims(C.byref(p), C.byref(na), C.byref(ns))
    if st != _abi.CSM_OK:
        raise CsmError(st, "invalid window parameters")
    return na.value, ns.value


# ---------------------------------------------------------------------------
# Reference-interface mirror
# ---------------------------------------------------------------------------

class BasedCorrelationScanMatch:
    """Mirror of BasedCorrelationScanMatch (correlate_scan_matcher.h:766-1036).

    ScanMatch(map, range_data, param, current_pose, cov_matrix) -> response;
    current_pose (world, 3) and cov_matrix (3x3) are updated in place exactly
    where the reference updates them.
    """

    def __init__(self, context: Context | None = None):
        self.ctx = context or Context(0)

    def ScanMatch(self, map_: ScanMatchMap, range_data: RangeDataContainer2d, param,
                  current_pose: np.ndarray, cov_matrix: np.ndarray) -> float:
        self.ctx.set_grid(map_)
        return self.ctx.scan_match(range_data.points, param, current_pose, cov_matrix.reshape(-1))


class BasedOptimizeScanMatch:
    """Mirror of BasedOptimizeScanMatch (optimize_scan_matcher.h:60-237).

    ScanMatch(map, range_data, param, best_pose) -> cost; best_pose (world, 3)
    is updated in place unless the reference's early returns apply.
    """

    def __init__(self, context: Context | None = None):
        self.ctx = context or Context(0)

    def ScanMatch(self, map_: ScanMatchMap, range_data: RangeDataContainer2d, param,
                  best_pose: np.ndarray) -> float:
        self.ctx.set_grid(map_)
        return self.ctx.optimize_scan_match(range_data.points, param, best_pose)


class ScanMatchers:
    """Mirror of ScanMatchers::ScanMatch (scan_matchers.h:179-289).

    With use_optimize_scan_match (ParamConfig default; both YAMLs turn it off)
    the Gauss-Newton matcher runs first on coarse_map with coarse_range_data
    and the correlative coarse level only when it fails (:205-242); every
    correlative level runs on fine_map with fine_range_data (:238,:249,:256).
    """

    def __init__(self, levels=SIM_YAML_LEVELS, context: Context | None = None,
                 use_optimize_scan_match: bool = False, optimize=SIM_YAML_OPTIMIZE,
                 optimize_failed_cost: float = 2.0, coarse_context: Context | None = None):
        self.levels = tuple(levels)
        self.ctx = context or Context(0)
        self.use_optimize_scan_match = use_optimize_scan_match
        self.optimize = optimize
        self.optimize_failed_cost = float(optimize_failed_cost)
        self.cctx = coarse_context or (Context(self.ctx.device) if use_optimize_scan_match else None)

    def ScanMatch(self, coarse_range_data, fine_range_data, coarse_map, fine_map,
                  best_pose: np.ndarray, cov_matrix: np.ndarray, use_fine_scan_match: bool = True) -> float:
        cov = cov_matrix.reshape(-1)
        if not self.use_optimize_scan_match:
            self.ctx.set_grid(fine_map)
            return self.ctx.scan_matchers(fine_range_data.points, self.levels, best_pose, cov,
                                          use_fine_scan_match)
        score, times = 0.0, 0
        process = best_pose.copy()
        self.cctx.set_grid(coarse_map)
        cost = self.cctx.optimize_scan_match(coarse_range_data.points, self.optimize, process)
        score = self.optimize_failed_cost / (cost + self.optimize_failed_cost)  # :211
        times += 1
        self.ctx.set_grid(fine_map)
        if not use_fine_scan_match or cost > self.optimize_failed_cost:  # :224-242
            score, times = 0.0, times - 1
            process[:] = best_pose
            score += self.ctx.scan_match(fine_range_data.points, self.levels[0], process, cov)
            times += 1
        best_pose[:] = process
        if use_fine_scan_match:
            for lv in self.levels[1:]:
                score += self.ctx.scan_match(fine_range_data.points, lv, process, cov)
                times += 1
        best_pose[:] = process
        return score / times


__all__ = [
    "Context", "CsmError", "ScanMatchMap", "RangeDataContainer2d", "BasedCorrelationScanMatch",
    "ScanMatchers", "CorrelationScanMatchParam", "SIM_YAML_LEVELS", "PARAM_CONFIG_LEVELS",
    "IN_CLASS_LEVELS", "FAST_PARAM", "BasedOptimizeScanMatch", "OptimizeScanMatchParam", "SIM_YAML_OPTIMIZE",
    "PARAM_CONFIG_OPTIMIZE", "CONFIG1_PARAM", "headline_levels", "window_dims",
    "cell_points", "COARSE", "FINE", "SUPER", "FAST", "kMapUnknownCellProb",
]
