"""GPU: the loop-closure search behind the C-ABI (include/csm_loop_closure.h,
csrc/csm_loop_closure.cpp): submaps sharded over the process's devices, the
MAX / MIN / SUM exchange over an in-process RCCL communicator. Checked
against the Python shard (roborts_csm.loop_closure.ShardedLoopClosure, whose
exchange is tested over gloo in test_loop_closure.py) and against the
oracle's per-submap argmax (oracle/csm_oracle.cpp)."""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import pyoracle as O  # noqa: E402


@pytest.fixture(scope="module")
def submaps(golden_dir):
    f1 = np.load(os.path.join(golden_dir, "f1_config1.npz"))
    rng = np.random.default_rng(43)
    base = np.stack([f1["grid"], np.roll(f1["grid"], 29, axis=0), np.roll(f1["grid"], -41, axis=1),
                     rng.choice(np.array([0.3, 0.5, 1.0], dtype=np.float32), size=f1["grid"].shape)])
    grids = np.concatenate([base, base[1:2], base[:1]])  # duplicates: cross-submap ties
    offsets = np.tile(np.asarray(f1["offset"], dtype=np.float64), (grids.shape[0], 1))
    offsets[3] += (0.35, -0.2)
    return f1, grids, offsets


def _devices():
    import ctypes as C
    n = C.c_int(0)
    hip = C.CDLL("libamdhip64.so")
    hip.hipGetDeviceCount(C.byref(n))
    return list(range(max(1, min(n.value, 8))))


@pytest.mark.parametrize("search", ["pyramid", "exhaustive"])
def test_capi_loop_closure_matches_python_shard_and_oracle(submaps, search):
    import roborts_csm
    from roborts_csm.loop_closure import DeviceLoopClosure, ShardedLoopClosure, world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    f1, grids, offsets = submaps
    res = float(f1["resolution"])
    p = CorrelationScanMatchParam(2.0, 0.05, math.pi / 2, 0.0349, 0.5, 100, 0, False, 0)
    pose = np.array(f1["init_pose"], dtype=np.float64)
    lc = DeviceLoopClosure(_devices())
    try:
        lc.set_submaps(grids, res, offsets, version=5)
        r = lc.match(f1["points"], p, pose, search=search)
    finally:
        lc.close()
    with roborts_csm.Context(0) as c:
        c.set_grid_stack(grids, res, version=5)
        r2 = ShardedLoopClosure(c, grids.shape[0], res, offsets, search=search).match(f1["points"], p, pose)
    assert (r.score, r.global_index, r.submap, r.x, r.y, r.angle) == \
           (r2.score, r2.global_index, r2.submap, r2.x, r2.y, r2.angle)
    na, ns = roborts_csm.window_dims(p)
    best = (-np.inf, None)
    for g in range(grids.shape[0]):
        s, flat = O.best_window(O.Map(grids[g], res, tuple(offsets[g])), f1["points"], p,
                                world_to_map(pose, res, offsets[g]))
        gi = g * na * ns * ns + flat
        if s > best[0] or (s == best[0] and gi < best[1]):
            best = (s, gi)
    assert (r.score, r.global_index) == best


def test_capi_loop_closure_world_pose(submaps):
    """The winner's world pose is GetWorldCoordsPose of its map-cell pose
    with its submap's offset (grid_map_base.h:83-87)."""
    from roborts_csm.loop_closure import DeviceLoopClosure
    from roborts_csm.params import CorrelationScanMatchParam
    f1, grids, offsets = submaps
    res = float(f1["resolution"])
    p = CorrelationScanMatchParam(1.0, 0.05, 0.3, 0.0349, 0.5, 100, 0, False, 0)
    lc = DeviceLoopClosure([0])
    try:
        lc.set_submaps(grids, res, offsets, version=1)
        r = lc.match(f1["points"], p, f1["init_pose"])
        s = 1.0 / res
        tx, ty = s * offsets[r.submap][0], s * offsets[r.submap][1]
        inv_a = s * (1.0 / (s * s - 0.0 * 0.0))
        want = [inv_a * r.x + -(inv_a * tx), inv_a * r.y + -(inv_a * ty), r.angle]
        assert list(lc.last_pose_world) == want
    finally:
        lc.close()
