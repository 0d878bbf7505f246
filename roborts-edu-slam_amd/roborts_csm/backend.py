"""The back-end's scan-match service (include/csm_backend.h).

Python mirror of SlamProcessor::ScanMatchInterface
(slam/slam_processor.cpp:250-326), the callback the pose graph calls for
near-chain links and loop closure (pose_graph/range_scan_pose_graph.cpp:
120-167, 299-355): `ScanMatchService.ScanMatchInterface(...)` is one call,
`scan_match_jobs(...)` runs many as one GPU batch. Parameters default to
config/simulatin_param.yaml (ParamConfig defaults where the YAML is silent).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field, fields

import numpy as np

from . import _abi
from .params import SIM_YAML_LEVELS, SIM_YAML_OPTIMIZE, SIM_YAML_OPTIMIZE_FAILED_COST

_lib = _abi.load_library()
_dp = C.POINTER(C.c_double)


class CsmBackendParam(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "range_max", "gaussian_blur_offset", "map_resolution", "coarse_map_resolution", "coarse_map_deviation",
        "fine_map_resolution", "fine_map_deviation")] + [(n, C.c_int32) for n in (
            "coarse_map_use_blur", "fine_map_use_blur", "use_map_check_feedback", "map_check_point_num")] + [
        ("map_check_bound_tolerance", C.c_double), ("map_check_penalty_gain", C.c_double),
        ("levels", _abi.CsmParam * 3), ("use_optimize_scan_match", C.c_int32), ("reserved", C.c_int32),
        ("optimize_failed_cost", C.c_double), ("optimize", _abi.CsmOptimizeParam)]


class CsmBackendJob(C.Structure):
    _fields_ = [("points_m", _dp), ("n_points", C.c_int32), ("n_chain", C.c_int32),
                ("chain_ids", C.POINTER(C.c_int32)), ("use_fine_scan_match", C.c_int32), ("reserved", C.c_int32),
                ("pose", C.c_double * 3), ("cov", C.c_double * 9), ("score", C.c_double),
                ("map_penalty", C.c_double), ("optimize_cost", C.c_double)]


@dataclass
class BackEndParam:
    """config/simulatin_param.yaml (+ ParamConfig defaults, param_config.h)."""

    range_max: float = 10.0
    gaussian_blur_offset: float = 0.88
    map_resolution: float = 0.05
    coarse_map_resolution: float = 0.08
    coarse_map_deviation: float = 0.24
    fine_map_resolution: float = 0.01
    fine_map_deviation: float = 0.03
    coarse_map_use_blur: bool = True
    fine_map_use_blur: bool = True
    use_map_check_feedback: bool = True
    map_check_point_num: int = 100
    map_check_bound_tolerance: float = 2.5
    map_check_penalty_gain: float = 0.015
    levels: tuple = field(default=SIM_YAML_LEVELS)
    use_optimize_scan_match: bool = False
    optimize_failed_cost: float = SIM_YAML_OPTIMIZE_FAILED_COST
    optimize: object = SIM_YAML_OPTIMIZE

    def to_c(self) -> CsmBackendParam:
        c = CsmBackendParam()
        for f in fields(self):
            if f.name == "levels":
                for k, lv in enumerate(self.levels):
                    c.levels[k] = lv.to_c()
            elif f.name == "optimize":
                c.optimize = self.optimize.to_c()
            else:
                setattr(c, f.name, type(getattr(c, f.name))(getattr(self, f.name)))
        return c


@dataclass
class JobResult:
    pose: np.ndarray
    cov: np.ndarray
    score: float
    map_penalty: float
    optimize_cost: float


def make_jobs(queries, chains, poses, use_fine=True):
    """ctypes job array; keeps the numpy buffers alive on the array."""
    n = len(queries)
    arr = (CsmBackendJob * max(n, 1))()
    keep = []
    for j in range(n):
        q = np.ascontiguousarray(queries[j], dtype=np.float64).reshape(-1, 2)
        ch = np.ascontiguousarray(chains[j], dtype=np.int32)
        keep += [q, ch]
        arr[j].points_m = q.ctypes.data_as(_dp)
        arr[j].n_points = q.shape[0]
        arr[j].chain_ids = ch.ctypes.data_as(C.POINTER(C.c_int32))
        arr[j].n_chain = ch.size
        arr[j].use_fine_scan_match = 1 if use_fine else 0
        for k in range(3):
            arr[j].pose[k] = float(poses[j][k])
    arr._keep = keep
    return arr


def job_results(arr, n) -> list[JobResult]:
    return [JobResult(np.array(arr[j].pose[:]), np.array(arr[j].cov[:]).reshape(3, 3), arr[j].score,
                      arr[j].map_penalty, arr[j].optimize_cost) for j in range(n)]


class ScanMatchService:
    """Back-end scan matching on one GPU (slam_processor.cpp:250-326)."""

    COARSE_MAP, FINE_MAP = 0, 1

    def __init__(self, param: BackEndParam | None = None, device: int = 0):
        self.param = param or BackEndParam()
        self._cp = self.param.to_c()
        h = C.c_void_p()
        st = _lib.csm_backend_create(int(device), C.byref(self._cp), C.byref(h))
        if st != _abi.CSM_OK:
            raise RuntimeError(f"csm_backend_create(device={device}) failed with status {st}")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.csm_backend_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        if st != _abi.CSM_OK:
            raise RuntimeError(f"csm_backend: status {st}: {_lib.csm_backend_last_error(self._h).decode()}")

    def AddRangeData(self, points_m, sensor_pose) -> int:
        """SensorDataManager::AddSensorData + the multi-resolution copies."""
        pts = np.ascontiguousarray(points_m, dtype=np.float64).reshape(-1, 2)
        pose = np.ascontiguousarray(sensor_pose, dtype=np.float64)
        i = C.c_int32(-1)
        self._check(_lib.csm_backend_add_scan(self._h, pts.ctypes.data_as(_dp), pts.shape[0],
                                              pose.ctypes.data_as(_dp), C.byref(i)))
        return i.value

    def UpdateRangeData(self, range_id: int, sensor_pose):  # slam_processor.cpp:597-603
        pose = np.ascontiguousarray(sensor_pose, dtype=np.float64)
        self._check(_lib.csm_backend_set_scan_pose(self._h, int(range_id), pose.ctypes.data_as(_dp)))

    def scan_match_jobs(self, queries, chains, poses, current_pose, pub_map=None, use_fine=True):
        """Many ScanMatchInterface calls in one batch -> list of JobResult."""
        arr = make_jobs(queries, chains, poses, use_fine)
        cur = np.ascontiguousarray(current_pose, dtype=np.float64)
        pub = pub_map._h if pub_map is not None else None
        self._check(_lib.csm_backend_scan_match(self._h, pub, cur.ctypes.data_as(_dp), arr, len(queries)))
        return job_results(arr, len(queries))

    def ScanMatchInterface(self, range_data_m, range_id, best_pose, current_pose, pub_map=None,
                           use_fine_scan_match=True):
        """One call; best_pose (3,) is updated in place; returns (score, cov)."""
        r = self.scan_match_jobs([range_data_m], [range_id], [best_pose], current_pose, pub_map,
                                 use_fine_scan_match)[0]
        best_pose[:] = r.pose
        return r.score, r.cov

    def map(self, slot: int, which: int):
        from .frontend import _BorrowedMap
        h = C.c_void_p()
        self._check(_lib.csm_backend_map(self._h, int(slot), int(which), C.byref(h)))
        if not h.value:
            raise RuntimeError("back-end map not created yet")
        return _BorrowedMap(h, self)
