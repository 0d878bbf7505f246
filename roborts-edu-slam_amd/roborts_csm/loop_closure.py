"""Loop-closure search sharded over GPUs.

The reference closes loops by matching a scan against the map around older
pose-chain candidates, one ScanMatchInterface call after another
(range_scan_pose_graph.cpp:299-355 TryCloseLoop, :120-167 LinkNearChains ->
slam_processor.cpp:301 -> ScanMatchers::ScanMatch). At loop-closure scale the
work is one query scan x many submaps x a large (x, y, theta) window, and the
answer is the single best candidate over all of them. Here:

* submaps are sharded by index across ranks, [r*S/G, (r+1)*S/G) resident on
  rank r (csm_set_grid_stack; no grid is replicated);
* each rank scores its submaps in one launch (csm_best_windows: argmax per
  window on the device) and reduces them to (best score, lowest global
  candidate index) -- global index = submap * n_cand + enumeration index;
* the one exchange step: all_reduce(MAX) of the score, then all_reduce(MIN)
  of the index among the ranks that hold that score, then the winner's
  (x, y, theta) from its owner (all_reduce(SUM) of a one-hot row). Over
  RCCL ("nccl") these are three 8-byte-scale collectives; the result does
  not depend on the rank count or order.

The scorer is anything with ``best_windows(points, param, grid_index,
centers) -> (scores, flat, x, y, angle)`` (search="exhaustive") or
``search_windows(points, param, grid_index, centers) -> (best, window,
stats)`` (search="pyramid", the admissible multi-resolution branch and
bound of csrc/csm_pyramid.hip: same answer, a fraction of the scorings):
the HIP context (roborts_csm.Context) in production.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import window_dims


def shard_range(n_submaps: int, rank: int, world: int) -> tuple[int, int]:
    """Submaps [lo, hi) of `rank` (contiguous, sizes differ by at most one)."""
    q, r = divmod(n_submaps, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def world_to_map(pose_world, resolution: float, offset) -> np.ndarray:
    """GridMapBase::GetMapCoordsPose (grid_map_base.h:68-69,89-93): Eigen's
    Scaling(1/res) * Translation(offset), evaluated in its order."""
    s = 1.0 / resolution
    return np.array([s * pose_world[0] + s * offset[0], s * pose_world[1] + s * offset[1], pose_world[2]])


def worlds_to_map(pose_world, resolution: float, offsets) -> np.ndarray:
    """world_to_map for every submap offset at once (the same expressions,
    elementwise: s * x + s * offset_x, with s = 1 / resolution)."""
    s = 1.0 / resolution
    off = np.asarray(offsets, dtype=np.float64).reshape(-1, 2)
    out = np.empty((off.shape[0], 3))
    out[:, 0] = s * pose_world[0] + s * off[:, 0]
    out[:, 1] = s * pose_world[1] + s * off[:, 1]
    out[:, 2] = pose_world[2]
    return out


@dataclass
class LoopClosureResult:
    score: float
    global_index: int   # submap * n_cand + enumeration index; -1: nothing scored
    submap: int
    x: float            # map cells of `submap`
    y: float
    angle: float


class ShardedLoopClosure:
    """One rank's share of the submaps and the exchange that merges ranks."""

    def __init__(self, scorer, n_submaps: int, resolution: float, offsets: np.ndarray,
                 rank: int = 0, world: int = 1, group=None, device=None, search: str = "pyramid"):
        assert search in ("pyramid", "exhaustive")
        self.scorer = scorer
        self.search = search
        self.last_stats = None
        self.n_submaps = int(n_submaps)
        self.resolution = float(resolution)
        self.lo, self.hi = shard_range(self.n_submaps, rank, world)
        self.offsets = np.asarray(offsets, dtype=np.float64).reshape(-1, 2)  # this shard's submaps
        assert self.offsets.shape[0] == self.hi - self.lo
        self.rank, self.world, self.group, self.device = rank, world, group, device

    def local_best(self, points_cells, param, pose_world) -> LoopClosureResult:
        n_loc = self.hi - self.lo
        if n_loc == 0:
            return LoopClosureResult(-np.inf, -1, -1, 0.0, 0.0, 0.0)
        na, ns = window_dims(param)
        n_cand = na * ns * ns
        centers = worlds_to_map(pose_world, self.resolution, self.offsets)
        if self.search == "pyramid":
            b, w, self.last_stats = self.scorer.search_windows(points_cells, param, np.arange(n_loc), centers)
            return LoopClosureResult(float(b.score), int((self.lo + w) * n_cand + b.flat_index), self.lo + w,
                                     float(b.x), float(b.y), float(b.angle))
        sc, flat, x, y, a = self.scorer.best_windows(points_cells, param, np.arange(n_loc), centers)
        gidx = (np.arange(self.lo, self.hi, dtype=np.int64) * n_cand + flat.astype(np.int64))
        best = np.max(sc)
        k = int(np.argmin(np.where(sc == best, gidx, np.iinfo(np.int64).max)))
        return LoopClosureResult(float(sc[k]), int(gidx[k]), self.lo + k, float(x[k]), float(y[k]), float(a[k]))

    def match(self, points_cells, param, pose_world) -> LoopClosureResult:
        loc = self.local_best(points_cells, param, pose_world)
        if self.world == 1:
            return loc
        import torch
        import torch.distributed as dist
        dev = self.device if self.device is not None else "cpu"
        s = torch.tensor([loc.score], dtype=torch.float64, device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.MAX, group=self.group)
        mine = loc.global_index if (loc.global_index >= 0 and loc.score == float(s.item())) else np.iinfo(np.int64).max
        i = torch.tensor([mine], dtype=torch.int64, device=dev)
        dist.all_reduce(i, op=dist.ReduceOp.MIN, group=self.group)
        win = int(i.item())
        row = torch.zeros(4, dtype=torch.float64, device=dev)
        if win == loc.global_index:
            row[:] = torch.tensor([loc.submap, loc.x, loc.y, loc.angle], dtype=torch.float64)
        dist.all_reduce(row, op=dist.ReduceOp.SUM, group=self.group)
        r = row.cpu().numpy()
        return LoopClosureResult(float(s.item()), win, int(r[0]), float(r[1]), float(r[2]), float(r[3]))


class DeviceLoopClosure:
    """The same search and exchange behind the C-ABI (include/csm_loop_closure.h):
    one process, the submaps sharded over `devices`, an in-process RCCL
    communicator per device (ncclCommInitAll) carrying the MAX / MIN / SUM
    all-reduces. What the reference's C++ back end (TryCloseLoop,
    range_scan_pose_graph.cpp:299-355) would call; no torch involved."""

    def __init__(self, devices=(0,)):
        import ctypes as C
        from . import _lib
        self._C, self._lib = C, _lib
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        h = C.c_void_p()
        st = _lib.csm_loop_closure_create(devs.size, devs.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(h))
        if st != 0:
            msg = _lib.csm_loop_closure_last_error(h).decode() if h.value else "create failed"
            if h.value:
                _lib.csm_loop_closure_destroy(h)
            from . import CsmError
            raise CsmError(st, msg)
        self._h = h
        self.n_devices = devs.size

    def _check(self, st):
        if st != 0:
            from . import CsmError
            raise CsmError(st, self._lib.csm_loop_closure_last_error(self._h).decode())

    def set_submaps(self, grids: np.ndarray, resolution: float, offsets, version: int = -1):
        from ._abi import CsmMapInfo
        C = self._C
        g = np.ascontiguousarray(grids, dtype=np.float32)
        self._grids = g  # resident by host pointer: keep alive
        off = np.ascontiguousarray(offsets, dtype=np.float64).reshape(-1, 2)
        assert off.shape[0] == g.shape[0]
        info = CsmMapInfo(float(resolution), 0.0, 0.0, g.shape[2], g.shape[1], 0, 0)
        self._check(self._lib.csm_loop_closure_set_submaps(self._h, g.ctypes.data_as(C.c_void_p), g.shape[0],
                                                           C.byref(info), off.ctypes.data_as(C.POINTER(C.c_double)),
                                                           int(version)))

    def match(self, points_cells, param, pose_world, search: str = "pyramid") -> LoopClosureResult:
        from . import _as_param
        from ._abi import CsmLoopClosureResult
        C = self._C
        pts = np.ascontiguousarray(points_cells, dtype=np.float64).reshape(-1, 2)
        pose = np.ascontiguousarray(pose_world, dtype=np.float64)
        p = _as_param(param)
        r = CsmLoopClosureResult()
        self._check(self._lib.csm_loop_closure_match(self._h, pts.ctypes.data_as(C.POINTER(C.c_double)), pts.shape[0],
                                                     C.byref(p), pose.ctypes.data_as(C.POINTER(C.c_double)),
                                                     0 if search == "pyramid" else 1, C.byref(r)))
        self.last_pose_world = np.array(r.pose_world[:])
        self.last_n_devices = int(r.n_devices)
        self.last_search_ms, self.last_exchange_ms = float(r.search_ms), float(r.exchange_ms)
        return LoopClosureResult(r.score, r.global_index, r.submap, r.x, r.y, r.angle)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.csm_loop_closure_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
