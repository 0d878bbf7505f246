"""Device-resident SLAM front-end (include/csm_frontend.h).

Python mirror of the reference's SlamProcessor front-end
(slam/slam_processor.cpp:65-248): `SlamFrontEnd.process(points_m, odom)` runs
one scan through the 3-level GPU matcher, the GPU map check and the GPU map
updates. Parameters default to config/simulatin_param.yaml (ParamConfig
fields, param_config.h:40-118, for what the YAML leaves out).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field, fields

import numpy as np

from . import _abi
from .gridmap import OccuGridMap
from .params import SIM_YAML_LEVELS, SIM_YAML_OPTIMIZE, SIM_YAML_OPTIMIZE_FAILED_COST

_lib = _abi.load_library()


class CsmFrontendParam(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "range_max", "init_map_size", "map_offset_x", "map_offset_y", "map_extend_factor", "gaussian_blur_offset",
        "map_resolution", "map_update_free_factor", "map_update_occu_factor", "map_occu_threshold",
        "map_min_passthrough", "coarse_map_resolution", "coarse_map_deviation", "fine_map_resolution",
        "fine_map_deviation")] + [(n, C.c_int32) for n in (
            "coarse_map_use_blur", "fine_map_use_blur", "use_odometry", "use_map_check_feedback",
            "map_check_point_num", "use_map_update_move_check")] + [(n, C.c_double) for n in (
                "map_check_bound_tolerance", "map_check_penalty_gain", "map_update_score_threshold",
                "map_update_distance_threshold", "map_update_angle_threshold")] + [
        ("levels", _abi.CsmParam * 3), ("use_optimize_scan_match", C.c_int32), ("reserved", C.c_int32),
        ("optimize_failed_cost", C.c_double), ("optimize", _abi.CsmOptimizeParam)]


class CsmFrontendResult(C.Structure):
    _fields_ = [("pose", C.c_double * 3), ("match_pose", C.c_double * 3), ("cov", C.c_double * 9),
                ("score", C.c_double), ("map_penalty", C.c_double), ("optimize_cost", C.c_double),
                ("data_index", C.c_int32),
                ("matched", C.c_int32), ("map_updated", C.c_int32), ("pose_accepted", C.c_int32)]


@dataclass
class FrontEndParam:
    """config/simulatin_param.yaml (+ ParamConfig defaults, param_config.h)."""

    range_max: float = 10.0                 # worlds/willow-pr2-5cm.world:7-13 Hokuyo
    init_map_size: float = 3.0
    map_offset_x: float = 0.5
    map_offset_y: float = 0.5
    map_extend_factor: float = 0.2
    gaussian_blur_offset: float = 0.88
    map_resolution: float = 0.05
    map_update_free_factor: float = 0.0
    map_update_occu_factor: float = 0.0
    map_occu_threshold: float = 0.2
    map_min_passthrough: float = 4.0
    coarse_map_resolution: float = 0.08
    coarse_map_deviation: float = 0.24
    fine_map_resolution: float = 0.01
    fine_map_deviation: float = 0.03
    coarse_map_use_blur: bool = True
    fine_map_use_blur: bool = True
    use_odometry: bool = True
    use_map_check_feedback: bool = True
    map_check_point_num: int = 100
    use_map_update_move_check: bool = False  # param_config.h default
    map_check_bound_tolerance: float = 2.5
    map_check_penalty_gain: float = 0.015
    map_update_score_threshold: float = 0.48  # param_config.h default
    map_update_distance_threshold: float = 0.1
    map_update_angle_threshold: float = 0.01745 * 1
    levels: tuple = field(default=SIM_YAML_LEVELS)
    use_optimize_scan_match: bool = False    # simulatin_param.yaml:40 (ParamConfig default: true)
    optimize_failed_cost: float = SIM_YAML_OPTIMIZE_FAILED_COST
    optimize: object = SIM_YAML_OPTIMIZE     # OptimizeScanMatchParam

    def to_c(self) -> CsmFrontendParam:
        c = CsmFrontendParam()
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
class FrontEndResult:
    pose: np.ndarray
    match_pose: np.ndarray
    cov: np.ndarray
    score: float
    map_penalty: float
    optimize_cost: float
    data_index: int
    matched: bool
    map_updated: bool
    pose_accepted: bool

    @staticmethod
    def from_c(r) -> "FrontEndResult":
        return FrontEndResult(np.array(r.pose[:]), np.array(r.match_pose[:]), np.array(r.cov[:]), r.score,
                              r.map_penalty, r.optimize_cost, r.data_index, bool(r.matched), bool(r.map_updated),
                              bool(r.pose_accepted))


class _BorrowedMap(OccuGridMap):
    """A map owned by the front-end (no destroy)."""

    def __init__(self, handle, owner):
        self._h = handle
        self._owner = owner
        self.kind = None
        self.device = owner.device

    def close(self):
        self._h = None


class SlamFrontEnd:
    """SlamProcessor front-end on one GPU (slam_processor.cpp:65-248)."""

    PUB_MAP, COARSE_MAP, FINE_MAP = 0, 1, 2

    def __init__(self, param: FrontEndParam | None = None, device: int = 0):
        self.param = param or FrontEndParam()
        self._cp = self.param.to_c()
        h = C.c_void_p()
        st = _lib.csm_frontend_create(int(device), C.byref(self._cp), C.byref(h))
        if st != _abi.CSM_OK:
            raise RuntimeError(f"csm_frontend_create(device={device}) failed with status {st}")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.csm_frontend_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, points_m, odom_pose) -> FrontEndResult:
        pts = np.ascontiguousarray(points_m, dtype=np.float64).reshape(-1, 2)
        od = np.ascontiguousarray(odom_pose, dtype=np.float64)
        r = CsmFrontendResult()
        st = _lib.csm_frontend_process(self._h, pts.ctypes.data_as(C.POINTER(C.c_double)), pts.shape[0],
                                       od.ctypes.data_as(C.POINTER(C.c_double)), C.byref(r))
        if st != _abi.CSM_OK:
            raise RuntimeError(f"csm_frontend_process: status {st}: {_lib.csm_frontend_last_error(self._h).decode()}")
        return FrontEndResult.from_c(r)

    def last_phases(self) -> dict:
        """Host wall time (ms) of the last process() call's phases
        (csm_frontend_last_phases): prepare, match, map_check, update_map and
        the latter's three maps."""
        out = np.zeros(7)
        _lib.csm_frontend_last_phases(self._h, out.ctypes.data_as(C.POINTER(C.c_double)))
        return dict(zip(("prepare", "match", "map_check", "update_map", "update_pub", "update_coarse", "update_fine"),
                        (float(x) for x in out)))

    def map(self, which: int) -> OccuGridMap:
        h = C.c_void_p()
        st = _lib.csm_frontend_map(self._h, int(which), C.byref(h))
        if st != _abi.CSM_OK or not h.value:
            raise RuntimeError("front-end map not available (no scan processed yet?)")
        return _BorrowedMap(h, self)

    def matcher(self):
        """The front end's scan-matcher context (borrowed): set_profiling /
        kernel_stats of the matches process() runs."""
        from . import Context
        h = C.c_void_p()
        st = _lib.csm_frontend_matcher(self._h, C.byref(h))
        if st != 0:
            raise RuntimeError(f"csm_frontend_matcher failed ({st})")
        return Context.borrow(h, self)

    def correct_pose_and_map(self, ids, poses) -> None:
        """SlamProcessor::CorrectPoseAndMap (slam/slam_processor.cpp:329-370):
        corrected world poses for kept scans `ids`, then the three maps are
        rebuilt on the device from every kept scan."""
        i = np.ascontiguousarray(ids, dtype=np.int32)
        p = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 3)
        assert p.shape[0] == i.size
        st = _lib.csm_frontend_correct_pose_and_map(self._h, i.size, i.ctypes.data_as(C.POINTER(C.c_int32)),
                                                    p.ctypes.data_as(C.POINTER(C.c_double)))
        if st != _abi.CSM_OK:
            raise RuntimeError(f"csm_frontend_correct_pose_and_map: status {st}: "
                               f"{_lib.csm_frontend_last_error(self._h).decode()}")

    def kept_poses(self) -> np.ndarray:
        n = C.c_int32(0)
        _lib.csm_frontend_kept_scans(self._h, C.byref(n), None)
        out = np.zeros((max(n.value, 1), 3))
        _lib.csm_frontend_kept_scans(self._h, C.byref(n), out.ctypes.data_as(C.POINTER(C.c_double)))
        return out[:n.value]
