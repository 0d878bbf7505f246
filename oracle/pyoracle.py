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
