"""Device-resident occupancy-grid maps (include/csm_gridmap.h).

Python mirror of the reference's OccuGridMap for the maps the scan matcher
reads and checks against:

  OccuGridMap(..., kind=PROBABILITY_CELL)  ~ ScanMatchMap = ProbCellMap (map/slam_map.h:32-36)
  OccuGridMap(..., kind=COUNT_CELL)        ~ PubMap = CountCellMap
  UpdateMapByRange                         ~ map/occu_grid_map.h:258-329
  InitMapWithRangeVec                      ~ map/occu_grid_map.h:222-255
  MapFeedbackResponsePenalty               ~ map/occu_grid_map.h:331-392

Cells live in HBM and every per-cell update is a HIP kernel of
libroborts_csm.so; this module only moves arrays and fails loudly when the
library or the device is missing.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import COUNT_CELL, PROBABILITY_CELL, CsmGridmapState

_lib = _abi.load_library()

kDefaultCellProb = np.float32(0.5)  # map/grid_map_cell.h:30


class GridMapError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"csm_gridmap status {status}: {msg}")
        self.status = status


def _d(a, shape=None) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a if shape is None else a.reshape(shape)


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class OccuGridMap:
    """One csm_gridmap (OccuGridMap<CellType, CellFunctions>, occu_grid_map.h:194-603)."""

    def __init__(self, resolution: float, size, offset, deviation: float = 0.0,
                 default_cell_prob: float = float(kDefaultCellProb), kind: int = PROBABILITY_CELL,
                 device: int = 0):
        h = C.c_void_p()
        st = _lib.csm_gridmap_create(int(device), int(kind), float(resolution), int(size[0]), int(size[1]),
                                     float(offset[0]), float(offset[1]), float(deviation),
                                     C.c_float(default_cell_prob), C.byref(h))
        if st != _abi.CSM_OK:
            raise GridMapError(st, f"csm_gridmap_create(device={device}) failed (no usable HIP device?)")
        self._h = h
        self.kind = kind
        self.device = device

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.csm_gridmap_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def _check(self, st: int):
        if st != _abi.CSM_OK:
            raise GridMapError(st, _lib.csm_gridmap_last_error(self._h).decode())

    # -- setters (occu_grid_map.h:413-439, grid_map_base.h:175-179,275-279) --
    def set_options(self, use_auto_map_resize: bool = True, just_update_occu: bool = False,
                    cell_occu_prob_offset: float = 0.72, extend_factor: float = 1.0):
        self._check(_lib.csm_gridmap_set_options(self._h, int(use_auto_map_resize), int(just_update_occu),
                                                 float(cell_occu_prob_offset), float(extend_factor)))

    def set_cell_params(self, update_free_factor: float, update_occu_factor: float,
                        occu_threshold: float = 0.5, min_pass: float = 2.0):
        self._check(_lib.csm_gridmap_set_cell_params(self._h, C.c_float(update_free_factor),
                                                     C.c_float(update_occu_factor), C.c_float(occu_threshold),
                                                     C.c_float(min_pass)))

    def set_map_offset(self, offset):
        self._check(_lib.csm_gridmap_set_map_offset(self._h, float(offset[0]), float(offset[1])))

    def Reset(self):
        self._check(_lib.csm_gridmap_reset(self._h))

    def UpdateBound(self, min_bound, max_bound) -> bool:
        """GridMapBase::UpdateBound (grid_map_base.h:247-264); False when the map grew."""
        inside = C.c_int32(0)
        self._check(_lib.csm_gridmap_update_bound(self._h, float(min_bound[0]), float(min_bound[1]),
                                                  float(max_bound[0]), float(max_bound[1]), C.byref(inside)))
        return bool(inside.value)

    # -- reference entry points -------------------------------------------------
    def UpdateMapByRange(self, points_cells, sensor_pose, use_blur: bool = False, origin=(0.0, 0.0)) -> bool:
        pts = _d(points_cells, (-1, 2))
        o, w = _d(origin), _d(sensor_pose)
        up = C.c_int32(0)
        self._check(_lib.csm_gridmap_update_by_range(self._h, _dp(pts), pts.shape[0], _dp(o), _dp(w),
                                                     int(use_blur), C.byref(up)))
        return bool(up.value)

    def InitMapWithRangeVec(self, scans, sensor_poses, use_blur: bool = False, use_reset_speedup: bool = False,
                            origins=None):
        scans = [_d(s, (-1, 2)) for s in scans]
        pts = np.ascontiguousarray(np.concatenate(scans)) if scans else np.zeros((0, 2))
        off = np.zeros(len(scans) + 1, dtype=np.int64)
        off[1:] = np.cumsum([s.shape[0] for s in scans])
        poses = _d(sensor_poses, (-1, 3))
        og = None if origins is None else _d(origins, (-1, 2))
        self._check(_lib.csm_gridmap_init_with_range_vec(
            self._h, len(scans), _dp(pts), off.ctypes.data_as(C.POINTER(C.c_int64)),
            None if og is None else _dp(og), _dp(poses), int(use_blur), int(use_reset_speedup)))

    def MapFeedbackResponsePenalty(self, points_cells, best_pose, check_point_num: int, bound_tolerance: float,
                                   penalty_gain: float, use_blur: bool = False, origin=(0.0, 0.0)) -> float:
        pts = _d(points_cells, (-1, 2))
        o, w = _d(origin), _d(best_pose)
        out = C.c_double(0.0)
        self._check(_lib.csm_gridmap_feedback_penalty(self._h, _dp(pts), pts.shape[0], _dp(o), _dp(w),
                                                      int(check_point_num), float(bound_tolerance),
                                                      float(penalty_gain), int(use_blur), C.byref(out)))
        return out.value

    # -- getters ---------------------------------------------------------------------
    def state(self) -> CsmGridmapState:
        st = CsmGridmapState()
        self._check(_lib.csm_gridmap_get_state(self._h, C.byref(st)))
        return st

    def GetSizeX(self) -> int:
        return self.state().size_x

    def GetSizeY(self) -> int:
        return self.state().size_y

    def map_update_index(self) -> int:
        return self.state().map_update_index

    def cells(self):
        """(prob, pass_count, hit_count, update_index, touched) as [size_y, size_x] host arrays."""
        s = self.state()
        sh = (s.size_y, s.size_x)
        prob, ps, hit = (np.empty(sh, dtype=np.float32) for _ in range(3))
        uidx = np.empty(sh, dtype=np.int32)
        touched = np.empty(sh, dtype=np.uint8)
        self._check(_lib.csm_gridmap_download(self._h, prob.ctypes.data, ps.ctypes.data, hit.ctypes.data,
                                              uidx.ctypes.data, touched.ctypes.data))
        return prob, ps, hit, uidx, touched

    def device_prob(self) -> int:
        p = C.c_void_p()
        self._check(_lib.csm_gridmap_device_prob(self._h, C.byref(p)))
        return int(p.value or 0)


def set_matcher_grid(ctx, m: OccuGridMap):
    """csm_set_grid_gridmap: the matcher context reads this map's probabilities."""
    ctx._check(_lib.csm_set_grid_gridmap(ctx._h, m.handle))
    ctx._grid_ref = m
