"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

*** TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT. ***
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline. PARITY UNPINNED: see
csm_oracle.cpp's header (the reference has no golden vectors for this path and
cannot be compiled here).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "liboracle.so")


class OracleParam(C.Structure):  # same layout as csm_param / CorrelationScanMatchParam
    _fields_ = [
        ("search_space_size", C.c_double),
        ("search_space_resolution", C.c_double),
        ("search_angle_offset", C.c_double),
        ("search_angle_resolution", C.c_double),
        ("response_threshold", C.c_double),
        ("use_point_size", C.c_int32),
        ("max_depth", C.c_int32),
        ("use_center_penalty", C.c_int32),
        ("type", C.c_int32),
    ]


class OracleMap(C.Structure):
    _fields_ = [
        ("cells", C.c_void_p),
        ("stride_floats", C.c_int64),
        ("size_x", C.c_int32),
        ("size_y", C.c_int32),
        ("resolution", C.c_double),
        ("offset_x", C.c_double),
        ("offset_y", C.c_double),
        ("update_index", C.c_int32),
        ("outside_value", C.c_float),
    ]


_dp = C.POINTER(C.c_double)
_i64p = C.POINTER(C.c_int64)


def _load():
    if not os.path.exists(LIB):
        raise OSError(f"{LIB} missing: run `make -C oracle`")
    lib = C.CDLL(LIB)
    sig = {
        "oracle_param_size": (C.c_int, []),
        "oracle_map_size": (C.c_int, []),
        "oracle_score_window": (C.c_int, [C.POINTER(OracleMap), _dp, C.c_int, C.c_void_p, _dp, _dp, C.c_int64]),
        "oracle_sorted_order": (C.c_int, [C.POINTER(OracleMap), _dp, C.c_int, C.c_void_p, _dp, _i64p, C.c_int64]),
        "oracle_scan_match": (C.c_double, [C.POINTER(OracleMap), _dp, C.c_int, C.c_void_p, _dp, _dp, _i64p, _i64p]),
        "oracle_scan_matchers": (C.c_double, [C.POINTER(OracleMap), _dp, C.c_int, C.c_void_p, C.c_int, _dp, _dp]),
        "oracle_scan_matchers_batch": (None, [C.POINTER(OracleMap), C.c_int, _dp, _i64p, C.c_void_p, C.c_int, _dp, _dp, _dp]),
        "oracle_world_to_map": (None, [C.POINTER(OracleMap), _dp, _dp]),
        "oracle_map_to_world": (None, [C.POINTER(OracleMap), _dp, _dp]),
        "oracle_best_window": (C.c_double, [C.POINTER(OracleMap), _dp, C.c_int, C.c_void_p, _dp, _i64p]),
        "oracle_std_sort_order": (None, [_dp, C.c_int64, _i64p]),
        "oracle_sincos_batch": (None, [_dp, C.c_int64, _dp, _dp]),
        "oracle_set_threads": (None, [C.c_int]),
    }
    for k, (r, a) in sig.items():
        f = getattr(lib, k)
        f.restype = r
        f.argtypes = a
    assert lib.oracle_param_size() == C.sizeof(OracleParam)
    assert lib.oracle_map_size() == C.sizeof(OracleMap)
    return lib


_lib = _load()


def _p(param) -> OracleParam:
    """Accept any object with the CorrelationScanMatchParam fields."""
    if isinstance(param, OracleParam):
        return param
    typ = getattr(param, "correlation_scan_match_type", getattr(param, "type", 0))
    return OracleParam(param.search_space_size, param.search_space_resolution,
                       param.search_angle_offset, param.search_angle_resolution,
                       param.response_threshold, int(param.use_point_size),
                       int(getattr(param, "max_depth", 0)), int(bool(param.use_center_penalty)),
                       int(typ))


class Map:
    """Oracle view of a grid (float32 [H,W] or AoS structured cells)."""

    def __init__(self, cells: np.ndarray, resolution: float, offset=(0.0, 0.0), update_index: int = 0,
                 outside: float = 0.3):
        if cells.dtype == np.float32:
            self._arr = np.ascontiguousarray(cells)
            stride = 1
        else:
            self._arr = np.ascontiguousarray(cells)
            stride = self._arr.dtype.itemsize // 4
        self.c = OracleMap(self._arr.ctypes.data, stride, self._arr.shape[1], self._arr.shape[0],
                           float(resolution), float(offset[0]), float(offset[1]), int(update_index),
                           float(np.float32(outside)))


def _pts(points):
    return np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 2)


def score_window(m: Map, points, param, center, n_out: int) -> np.ndarray:
    pts = _pts(points)
    out = np.empty(n_out)
    ctr = np.ascontiguousarray(center, dtype=np.float64)
    p = _p(param)
    st = _lib.oracle_score_window(C.byref(m.c), pts.ctypes.data_as(_dp), pts.shape[0], C.byref(p),
                                  ctr.ctypes.data_as(_dp), out.ctypes.data_as(_dp), n_out)
    assert st == 0
    return out


def sorted_order(m: Map, points, param, center, n_out: int) -> np.ndarray:
    pts = _pts(points)
    out = np.empty(n_out, dtype=np.int64)
    ctr = np.ascontiguousarray(center, dtype=np.float64)
    p = _p(param)
    st = _lib.oracle_sorted_order(C.byref(m.c), pts.ctypes.data_as(_dp), pts.shape[0], C.byref(p),
                                  ctr.ctypes.data_as(_dp), out.ctypes.data_as(_i64p), n_out)
    assert st == 0
    return out


def scan_match(m: Map, points, param, pose, cov):
    """Returns (response, pose', cov', argmax_flat, n_scored)."""
    pts = _pts(points)
    pose = np.array(pose, dtype=np.float64)
    cov = np.array(cov, dtype=np.float64).reshape(9)
    am, ns = C.c_int64(0), C.c_int64(0)
    p = _p(param)
    r = _lib.oracle_scan_match(C.byref(m.c), pts.ctypes.data_as(_dp), pts.shape[0], C.byref(p),
                               pose.ctypes.data_as(_dp), cov.ctypes.data_as(_dp), C.byref(am), C.byref(ns))
    return r, pose, cov, am.value, ns.value


def scan_matchers(m: Map, points, levels, pose, cov, use_fine: bool = True):
    pts = _pts(points)
    pose = np.array(pose, dtype=np.float64)
    cov = np.array(cov, dtype=np.float64).reshape(9)
    lv = (OracleParam * 3)(*[_p(l) for l in levels])
    r = _lib.oracle_scan_matchers(C.byref(m.c), pts.ctypes.data_as(_dp), pts.shape[0], lv,
                                  1 if use_fine else 0, pose.ctypes.data_as(_dp), cov.ctypes.data_as(_dp))
    return r, pose, cov


def set_threads(n: int) -> None:
    """Threads for the candidate enumeration (OpenMP over theta; 1 = the
    reference's single-threaded loop). Results do not depend on it."""
    _lib.oracle_set_threads(int(n))


def scan_matchers_batch(m: Map, points, offsets, levels, poses, covs, use_fine: bool = True):
    pts = _pts(points)
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    n = off.size - 1
    poses = np.array(poses, dtype=np.float64).reshape(n, 3)
    covs = np.array(covs, dtype=np.float64).reshape(n, 9)
    scores = np.zeros(n)
    lv = (OracleParam * 3)(*[_p(l) for l in levels])
    _lib.oracle_scan_matchers_batch(C.byref(m.c), n, pts.ctypes.data_as(_dp), off.ctypes.data_as(_i64p), lv,
                                    1 if use_fine else 0, poses.ctypes.data_as(_dp), covs.ctypes.data_as(_dp),
                                    scores.ctypes.data_as(_dp))
    return scores, poses, covs


def world_to_map(m: Map, w):
    w = np.ascontiguousarray(w, dtype=np.float64)
    out = np.empty(3)
    _lib.oracle_world_to_map(C.byref(m.c), w.ctypes.data_as(_dp), out.ctypes.data_as(_dp))
    return out


def map_to_world(m: Map, p):
    p = np.ascontiguousarray(p, dtype=np.float64)
    out = np.empty(3)
    _lib.oracle_map_to_world(C.byref(m.c), p.ctypes.data_as(_dp), out.ctypes.data_as(_dp))
    return out


def best_window(m: Map, points, param, center):
    pts = _pts(points)
    ctr = np.ascontiguousarray(center, dtype=np.float64)
    f = C.c_int64(0)
    p = _p(param)
    s = _lib.oracle_best_window(C.byref(m.c), pts.ctypes.data_as(_dp), pts.shape[0], C.byref(p),
                                ctr.ctypes.data_as(_dp), C.byref(f))
    return s, f.value


def std_sort_order(keys) -> np.ndarray:
    """Permutation libstdc++'s std::sort(greater) applies to keys."""
    k = np.ascontiguousarray(keys, dtype=np.float64)
    out = np.empty(k.size, dtype=np.int64)
    _lib.oracle_std_sort_order(k.ctypes.data_as(_dp), k.size, out.ctypes.data_as(_i64p))
    return out


def sincos_batch(x):
    """(sin x, cos x) from the host libm's sincos, element by element."""
    a = np.ascontiguousarray(x, dtype=np.float64)
    s = np.empty_like(a)
    c = np.empty_like(a)
    _lib.oracle_sincos_batch(a.ctypes.data_as(_dp), a.size, s.ctypes.data_as(_dp), c.ctypes.data_as(_dp))
    return s, c


# ---- occupancy-grid map building (map_oracle.cpp) ----
PROBABILITY_CELL, COUNT_CELL = 0, 1
_fp = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)
for _k, (_r, _a) in {
    "oracle_gridmap_create": (C.c_void_p, [C.c_int, C.c_double, C.c_int, C.c_int, C.c_double, C.c_double,
                                           C.c_double, C.c_float]),
    "oracle_gridmap_destroy": (None, [C.c_void_p]),
    "oracle_gridmap_set_options": (None, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double]),
    "oracle_gridmap_set_cell_params": (None, [C.c_void_p, C.c_float, C.c_float, C.c_float, C.c_float]),
    "oracle_gridmap_set_map_offset": (None, [C.c_void_p, C.c_double, C.c_double]),
    "oracle_gridmap_reset": (None, [C.c_void_p]),
    "oracle_gridmap_update_by_range": (C.c_int, [C.c_void_p, _dp, C.c_int, _dp, _dp, C.c_int]),
    "oracle_gridmap_init_with_range_vec": (None, [C.c_void_p, _dp, _i64p, C.c_int, _dp, _dp, C.c_int, C.c_int]),
    "oracle_gridmap_feedback_penalty": (C.c_double, [C.c_void_p, _dp, C.c_int, _dp, _dp, C.c_int, C.c_double,
                                                     C.c_double, C.c_int]),
    "oracle_gridmap_info": (None, [C.c_void_p, _i32p, _dp]),
    "oracle_gridmap_cells": (None, [C.c_void_p, _fp, _fp, _fp, _i32p]),
    "oracle_gridmap_touched": (None, [C.c_void_p, _u8p]),
    "oracle_gridmap_kernel": (C.c_int, [C.c_void_p, _dp, C.c_int]),
    "oracle_bresenham": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, _i32p, C.c_int]),
}.items():
    _f = getattr(_lib, _k)
    _f.restype, _f.argtypes = _r, _a


def _d(a, n=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a


class GridMap:
    """Oracle OccuGridMap<ProbabilityCell | CountCell> (map_oracle.cpp)."""

    def __init__(self, kind: int, resolution: float, size, offset, deviation: float = 0.0,
                 default_prob: float = 0.5):
        self.h = _lib.oracle_gridmap_create(kind, resolution, int(size[0]), int(size[1]), float(offset[0]),
                                            float(offset[1]), deviation, default_prob)

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            _lib.oracle_gridmap_destroy(h)
            self.h = None

    def set_options(self, auto_resize=True, just_update_occu=False, occu_offset=0.72, extend_factor=1.0):
        _lib.oracle_gridmap_set_options(self.h, int(auto_resize), int(just_update_occu), occu_offset, extend_factor)

    def set_cell_params(self, free_factor, occu_factor, occu_threshold=0.5, min_pass=2.0):
        _lib.oracle_gridmap_set_cell_params(self.h, free_factor, occu_factor, occu_threshold, min_pass)

    def set_map_offset(self, ox, oy):
        _lib.oracle_gridmap_set_map_offset(self.h, ox, oy)

    def reset(self):
        _lib.oracle_gridmap_reset(self.h)

    def update_by_range(self, points, pose, origin=(0.0, 0.0), use_blur=False) -> bool:
        p = _pts(points)
        o, w = _d(origin), _d(pose)
        return bool(_lib.oracle_gridmap_update_by_range(self.h, p.ctypes.data_as(_dp), p.shape[0],
                                                        o.ctypes.data_as(_dp), w.ctypes.data_as(_dp),
                                                        int(use_blur)))

    def init_with_range_vec(self, scans, poses, origins=None, use_blur=False, speedup=False):
        pts = np.concatenate([_pts(s) for s in scans]) if scans else np.zeros((0, 2))
        pts = np.ascontiguousarray(pts)
        off = np.zeros(len(scans) + 1, dtype=np.int64)
        off[1:] = np.cumsum([_pts(s).shape[0] for s in scans])
        ps = _d(np.asarray(poses, dtype=np.float64).reshape(-1, 3))
        og = _d(np.zeros((len(scans), 2)) if origins is None else np.asarray(origins).reshape(-1, 2))
        _lib.oracle_gridmap_init_with_range_vec(self.h, pts.ctypes.data_as(_dp), off.ctypes.data_as(_i64p),
                                                len(scans), og.ctypes.data_as(_dp), ps.ctypes.data_as(_dp),
                                                int(use_blur), int(speedup))

    def feedback_penalty(self, points, best_pose, check_point_num, bound_tolerance, penalty_gain,
                         origin=(0.0, 0.0), use_blur=False) -> float:
        p = _pts(points)
        o, w = _d(origin), _d(best_pose)
        return _lib.oracle_gridmap_feedback_penalty(self.h, p.ctypes.data_as(_dp), p.shape[0],
                                                    o.ctypes.data_as(_dp), w.ctypes.data_as(_dp),
                                                    int(check_point_num), bound_tolerance, penalty_gain,
                                                    int(use_blur))

    def info(self) -> dict:
        ints = np.zeros(8, dtype=np.int32)
        dbl = np.zeros(7)
        _lib.oracle_gridmap_info(self.h, ints.ctypes.data_as(_i32p), dbl.ctypes.data_as(_dp))
        return {"size_x": int(ints[0]), "size_y": int(ints[1]), "map_update_index": int(ints[2]),
                "cur_update_index": int(ints[3]), "half_kernel": int(ints[4]), "n_update_points": int(ints[5]),
                "blur_states": bool(ints[6]), "kind": int(ints[7]), "resolution": dbl[0],
                "offset": (dbl[1], dbl[2]), "bound": tuple(dbl[3:7])}

    def cells(self):
        """(prob, pass, hit, update_index) as [size_y, size_x] arrays."""
        inf = self.info()
        n = inf["size_x"] * inf["size_y"]
        prob, ps, hit = (np.zeros(n, dtype=np.float32) for _ in range(3))
        uidx = np.zeros(n, dtype=np.int32)
        _lib.oracle_gridmap_cells(self.h, prob.ctypes.data_as(_fp), ps.ctypes.data_as(_fp), hit.ctypes.data_as(_fp),
                                  uidx.ctypes.data_as(_i32p))
        sh = (inf["size_y"], inf["size_x"])
        return prob.reshape(sh), ps.reshape(sh), hit.reshape(sh), uidx.reshape(sh)

    def touched(self) -> np.ndarray:
        inf = self.info()
        f = np.zeros(inf["size_x"] * inf["size_y"], dtype=np.uint8)
        _lib.oracle_gridmap_touched(self.h, f.ctypes.data_as(_u8p))
        return f

    def kernel(self) -> np.ndarray:
        out = np.zeros(441)
        n = _lib.oracle_gridmap_kernel(self.h, out.ctypes.data_as(_dp), out.size)
        return out[:n]


def bresenham(x0, y0, x1, y1) -> np.ndarray:
    cap = abs(x1 - x0) + abs(y1 - y0) + 2
    out = np.zeros(2 * cap, dtype=np.int32)
    n = _lib.oracle_bresenham(x0, y0, x1, y1, out.ctypes.data_as(_i32p), cap)
    return out[:2 * n].reshape(n, 2)


# ---- SlamProcessor front-end (map_oracle.cpp oracle_frontend_*) ----------------
for _k, (_r, _a) in {
    "oracle_frontend_create": (C.c_void_p, [C.c_void_p]),
    "oracle_frontend_destroy": (None, [C.c_void_p]),
    "oracle_frontend_param_size": (C.c_int, []),
    "oracle_frontend_result_size": (C.c_int, []),
    "oracle_frontend_map": (C.c_void_p, [C.c_void_p, C.c_int]),
    "oracle_frontend_process": (C.c_int, [C.c_void_p, _dp, C.c_int, _dp, C.c_void_p]),
    "oracle_frontend_correct": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int32), _dp]),
}.items():
    _f = getattr(_lib, _k)
    _f.restype, _f.argtypes = _r, _a


class _FrontEndMap(GridMap):
    def __init__(self, h, owner):  # borrowed OMap* (owned by the front-end)
        self.h = h
        self._owner = owner

    def __del__(self):
        pass


class FrontEnd:
    """Oracle SlamProcessor front-end; param / result are ctypes structures with
    the csm_frontend_param / csm_frontend_result layouts."""

    def __init__(self, c_param):
        assert _lib.oracle_frontend_param_size() == C.sizeof(c_param)
        self._p = c_param
        self.h = _lib.oracle_frontend_create(C.byref(c_param))

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            _lib.oracle_frontend_destroy(h)
            self.h = None

    def process(self, points_m, odom, result):
        assert _lib.oracle_frontend_result_size() == C.sizeof(result)
        p = _pts(points_m)
        o = _d(odom)
        _lib.oracle_frontend_process(self.h, p.ctypes.data_as(_dp), p.shape[0], o.ctypes.data_as(_dp),
                                     C.byref(result))
        return result

    def map(self, which: int) -> GridMap:
        return _FrontEndMap(_lib.oracle_frontend_map(self.h, which), self)

    def correct_pose_and_map(self, ids, poses) -> None:
        """SlamProcessor::CorrectPoseAndMap (slam_processor.cpp:329-370)."""
        i = np.ascontiguousarray(ids, dtype=np.int32)
        p = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 3)
        assert p.shape[0] == i.size
        st = _lib.oracle_frontend_correct(self.h, i.size, i.ctypes.data_as(C.POINTER(C.c_int32)),
                                          p.ctypes.data_as(_dp))
        if st != 0:
            raise ValueError("corrected id beyond the kept scans")


# ---- BasedOptimizeScanMatch (opt_oracle.cpp) ----------------------------------
class OracleOptParam(C.Structure):  # same layout as csm_optimize_param
    _fields_ = [
        ("iterate_max_times", C.c_int32),
        ("reserved", C.c_int32),
        ("cost_decrease_threshold", C.c_double),
        ("cost_min_threshold", C.c_double),
        ("max_update_distance", C.c_double),
        ("max_update_angle", C.c_double),
    ]


for _k, (_r, _a) in {
    "oracle_optimize_param_size": (C.c_int, []),
    "oracle_optimize_scan_match": (C.c_double, [C.POINTER(OracleMap), _dp, C.c_int, C.c_void_p, _dp,
                                                C.POINTER(C.c_int)]),
    "oracle_optimize_update_cost": (C.c_double, [C.POINTER(OracleMap), _dp, C.c_int, _dp, _dp, _dp]),
    "oracle_ldlt_solve": (None, [_dp, _dp, _dp]),
}.items():
    getattr(_lib, _k).restype = _r
    getattr(_lib, _k).argtypes = _a
assert _lib.oracle_optimize_param_size() == C.sizeof(OracleOptParam)


def _op(param) -> OracleOptParam:
    if isinstance(param, OracleOptParam):
        return param
    return OracleOptParam(int(param.iterate_max_times), 0, param.cost_decrease_threshold, param.cost_min_threshold,
                          param.max_update_distance, param.max_update_angle)


def optimize_scan_match(m: Map, points, param, pose):
    """BasedOptimizeScanMatch::ScanMatch -> (cost, pose', iterations)."""
    pts = _pts(points)
    pose = np.array(pose, dtype=np.float64)
    it = C.c_int(0)
    p = _op(param)
    cost = _lib.oracle_optimize_scan_match(C.byref(m.c), pts.ctypes.data_as(_dp), pts.shape[0], C.byref(p),
                                           pose.ctypes.data_as(_dp), C.byref(it))
    return cost, pose, it.value


def optimize_update_cost(m: Map, points, est_map):
    """One UpdateCost at a map-cell pose -> (normalised cost, H (3x3), b)."""
    pts = _pts(points)
    est = np.ascontiguousarray(est_map, dtype=np.float64)
    H = np.zeros(9)
    b = np.zeros(3)
    c = _lib.oracle_optimize_update_cost(C.byref(m.c), pts.ctypes.data_as(_dp), pts.shape[0],
                                         est.ctypes.data_as(_dp), H.ctypes.data_as(_dp), b.ctypes.data_as(_dp))
    return c, H.reshape(3, 3), b


def ldlt_solve(H, b):
    """Eigen 3.3 LDLT<Matrix3d>::solve restated (lower triangle of H read)."""
    h = np.ascontiguousarray(H, dtype=np.float64).reshape(9)
    bb = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(3)
    _lib.oracle_ldlt_solve(h.ctypes.data_as(_dp), bb.ctypes.data_as(_dp), x.ctypes.data_as(_dp))
    return x


# ---- SlamProcessor::ScanMatchInterface (map_oracle.cpp oracle_backend_*) --------
for _k, (_r, _a) in {
    "oracle_backend_create": (C.c_void_p, [C.c_void_p]),
    "oracle_backend_destroy": (None, [C.c_void_p]),
    "oracle_backend_param_size": (C.c_int, []),
    "oracle_backend_job_size": (C.c_int, []),
    "oracle_backend_map": (C.c_void_p, [C.c_void_p, C.c_int, C.c_int]),
    "oracle_backend_add_scan": (C.c_int, [C.c_void_p, _dp, C.c_int, _dp]),
    "oracle_backend_set_scan_pose": (None, [C.c_void_p, C.c_int, _dp]),
    "oracle_backend_scan_match": (C.c_int, [C.c_void_p, C.c_void_p, _dp, C.c_void_p, C.c_int]),
}.items():
    _f = getattr(_lib, _k)
    _f.restype, _f.argtypes = _r, _a


class BackEnd:
    """Oracle back-end scan-match service; param / jobs are ctypes structures
    with the csm_backend_param / csm_backend_job layouts (roborts_csm.backend)."""

    def __init__(self, c_param):
        assert _lib.oracle_backend_param_size() == C.sizeof(c_param)
        self._p = c_param
        self.h = _lib.oracle_backend_create(C.byref(c_param))

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            _lib.oracle_backend_destroy(h)
            self.h = None

    def add_scan(self, points_m, pose) -> int:
        p, w = _pts(points_m), _d(pose)
        return _lib.oracle_backend_add_scan(self.h, p.ctypes.data_as(_dp), p.shape[0], w.ctypes.data_as(_dp))

    def set_scan_pose(self, i: int, pose):
        w = _d(pose)
        _lib.oracle_backend_set_scan_pose(self.h, int(i), w.ctypes.data_as(_dp))

    def scan_match(self, jobs, n_jobs: int, current_pose, pub_map: GridMap | None = None):
        assert _lib.oracle_backend_job_size() == C.sizeof(jobs[0])
        cur = _d(current_pose)
        _lib.oracle_backend_scan_match(self.h, pub_map.h if pub_map is not None else None, cur.ctypes.data_as(_dp),
                                       jobs, n_jobs)
        return jobs

    def map(self, slot: int, which: int) -> GridMap:
        return _FrontEndMap(_lib.oracle_backend_map(self.h, slot, which), self)
