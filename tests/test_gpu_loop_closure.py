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


def test_capi_failed_set_submaps_leaves_no_submaps(submaps):
    """A set_submaps that fails part-way commits nothing: the next match
    fails with CSM_ERR_NO_GRID instead of searching a mix of old and new
    shards under the old ranges (csm_loop_closure.cpp)."""
    import ctypes as C

    from roborts_csm import CsmError
    from roborts_csm._abi import CSM_ERR_NO_GRID, CsmMapInfo
    from roborts_csm.loop_closure import DeviceLoopClosure
    from roborts_csm.params import CorrelationScanMatchParam
    f1, grids, offsets = submaps
    res = float(f1["resolution"])
    p = CorrelationScanMatchParam(1.0, 0.05, 0.3, 0.0349, 0.5, 100, 0, False, 0)
    lc = DeviceLoopClosure(_devices())
    try:
        lc.set_submaps(grids, res, offsets, version=1)
        lc.match(f1["points"], p, f1["init_pose"])
        bad = CsmMapInfo(res, 0.0, 0.0, -5, grids.shape[1], 0, 0)  # every shard's upload fails
        g = np.ascontiguousarray(grids)
        off = np.ascontiguousarray(offsets)
        st = lc._lib.csm_loop_closure_set_submaps(lc._h, g.ctypes.data_as(C.c_void_p), 2 * g.shape[0], C.byref(bad),
                                                  off.ctypes.data_as(C.POINTER(C.c_double)), 2)
        assert st != 0
        with pytest.raises(CsmError) as ei:
            lc.match(f1["points"], p, f1["init_pose"])
        assert ei.value.status == CSM_ERR_NO_GRID
        lc.set_submaps(grids, res, offsets, version=3)  # a good call restores service
        assert lc.match(f1["points"], p, f1["init_pose"]).submap >= 0
    finally:
        lc.close()


def test_calls_restore_the_callers_device(submaps):
    """Every C-ABI call selects its context's device and hands the caller's
    current device back (a host process must not be left on
    another GPU)."""
    import ctypes as C

    import roborts_csm
    from roborts_csm.loop_closure import DeviceLoopClosure
    from roborts_csm.params import CorrelationScanMatchParam
    hip = C.CDLL("libamdhip64.so")
    n = C.c_int(0)
    hip.hipGetDeviceCount(C.byref(n))
    last = n.value - 1
    cur = C.c_int(-1)
    hip.hipSetDevice(last)
    f1, grids, offsets = submaps
    p = CorrelationScanMatchParam(1.0, 0.05, 0.3, 0.0349, 0.5, 100, 0, False, 0)
    with roborts_csm.Context(0) as ctx:
        ctx.set_grid(roborts_csm.ScanMatchMap(f1["grid"], float(f1["resolution"]), tuple(f1["offset"])), force=True)
        pose = np.array(f1["init_pose"], dtype=np.float64)
        ctx.scan_match(f1["points"], p, pose, np.eye(3).reshape(9).copy())
        hip.hipGetDevice(C.byref(cur))
        assert cur.value == last
    lc = DeviceLoopClosure([0])
    try:
        lc.set_submaps(grids, float(f1["resolution"]), offsets, version=1)
        lc.match(f1["points"], p, f1["init_pose"])
        hip.hipGetDevice(C.byref(cur))
        assert cur.value == last
    finally:
        lc.close()
        hip.hipSetDevice(0)


def test_bench_lc_capi_mode_runs():
    """bench.py --workload loop_closure --lc capi: one process through
    csm_loop_closure_* (in-process RCCL communicator over every visible
    device), the result line reports the library's n_devices."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--workload", "loop_closure", "--lc", "capi",
                        "--gpus", "1", "--submaps", "16", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["config"]["lc"] == "capi" and d["config"]["n_devices"] == 1 and d["value"] > 0
    assert d["result"]["submap"] >= 0


def test_bench_lc_leg_one_device():
    """The default line's config-3 leg (bench.py lc_leg: a child over every
    requested device through csm_loop_closure_*, RCCL exchange timed per
    query) at one device: ok, and equal to the one-device answer computed
    by a plain matcher context in the same child."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import tempfile
    detail = os.path.join(tempfile.mkdtemp(), "detail.json")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--workload", "plumbing", "--lc-leg",
                        "--gpus", "1", "--submaps", "24", "--lc-steps", "3", "--steps", "2", "--detail-json", detail],
                       capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    short = d["loop_closure_rccl"]  # the compact line's summary of the leg
    assert short["status"] == "ok" and short["n_devices"] == 1 and short["same_as_one_device"] is True, short
    with open(detail) as f:  # the whole leg: the side file
        leg = json.load(f)["loop_closure_rccl"]
    assert leg["status"] == "ok", leg
    assert leg["n_devices"] == 1 and leg["submaps_per_device"] == [24] and leg["steps"] == 3
    assert leg["verify"]["same_as_one_device"] is True, leg["verify"]
    assert leg["result"]["global_index"] == leg["verify"]["one_device"]["global_index"] >= 0
    assert leg["exchange_us"]["median"] > 0 and leg["ms_per_query"] > 0
