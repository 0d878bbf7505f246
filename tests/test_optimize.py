"""Gauss-Newton scan matcher (optimize_scan_matcher.h:68-221).

CPU: the oracle (oracle/opt_oracle.cpp) against the committed F6 fixture and
the independent pure-Python restatement (tests/opt_pyref.py), bit for bit;
its Eigen-LDLT restatement against numpy's solve (tolerance 1e-10 relative:
different algorithms) and on the degenerate cases; convergence on ray-cast
scans. GPU: csm_optimize_scan_match(_batch) against the oracle bit for bit
(cost, pose, iteration count), including the reference's early returns.

PARITY UNPINNED by the reference (no tests; Eigen absent, so the LDLT is
restated from Eigen 3.3's algorithm and pinned by the two restatements).
"""
import math
import os

import numpy as np
import pytest

import opt_pyref as R
import pyoracle as O


@pytest.fixture(scope="module")
def f6(golden_dir):
    return np.load(os.path.join(golden_dir, "f6_optimize.npz"))


@pytest.fixture(scope="module")
def f1(golden_dir):
    return np.load(os.path.join(golden_dir, "f1_config1.npz"))


def _prm(a):
    from roborts_csm.params import OptimizeScanMatchParam
    return OptimizeScanMatchParam(int(a[0]), float(a[1]), float(a[2]), float(a[3]), float(a[4]))


def _scans(f6):
    off = f6["offsets"]
    return [f6["points"][off[k]:off[k + 1]] for k in range(off.size - 1)]


def test_f6_oracle_reproduces_fixture(f1, f6):
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    for tag in ("sim", "cfg"):
        prm = _prm(f6[f"param_{tag}"])
        for k, pts in enumerate(_scans(f6)):
            c, p, it = O.optimize_scan_match(m, pts, prm, f6["init_poses"][k])
            assert c == f6[f"cost_{tag}"][k] and np.array_equal(p, f6[f"pose_{tag}"][k]), (tag, k)
            assert it == f6[f"iters_{tag}"][k]


def test_f6_independent_restatement(f1, f6):
    grid, res, off = f1["grid"], float(f1["resolution"]), tuple(float(v) for v in f1["offset"])
    prm = _prm(f6["param_sim"])
    for k, pts in enumerate(_scans(f6)[:3]):
        c, p, it = R.optimize_scan_match(grid, res, off, pts, prm, f6["init_poses"][k])
        assert c == f6["cost_sim"][k] and p == list(f6["pose_sim"][k]) and it == f6["iters_sim"][k], k


def test_update_cost_matches_restatement(f1, f6):
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    pts = _scans(f6)[0]
    est = O.world_to_map(m, f6["init_poses"][0])
    c, H, b = O.optimize_update_cost(m, pts, est)
    c2, H2, b2 = R.update_cost(f1["grid"], pts, list(est))
    assert c == c2 and np.array_equal(H, np.array(H2)) and np.array_equal(b, np.array(b2))
    assert np.array_equal(H, H.T)


def test_ldlt_restatement():
    rng = np.random.default_rng(5)
    for _ in range(200):
        A = rng.normal(size=(3, 3))
        H = A @ A.T + 1e-3 * np.eye(3)
        b = rng.normal(size=3)
        x = O.ldlt_solve(H, b)
        assert x.tolist() == R.ldlt_solve(H.tolist(), b.tolist())
        assert np.allclose(x, np.linalg.solve(H, b), rtol=1e-10, atol=1e-12)
    # pivoting order matters: a tiny leading diagonal is swapped away
    H = np.array([[1e-9, 0.0, 0.0], [0.0, 7.0, 1.0], [0.0, 1.0, 2.0]])
    assert np.allclose(O.ldlt_solve(H, [1.0, 2.0, 3.0]), np.linalg.solve(H, [1.0, 2.0, 3.0]))
    # all-zero H: Eigen stops at k = 0 and the pseudo-inverse zeroes everything
    assert O.ldlt_solve(np.zeros((3, 3)), [1.0, 2.0, 3.0]).tolist() == [0.0, 0.0, 0.0]
    # rank-deficient: the zero pivot row is zeroed, not divided
    H = np.diag([2.0, 0.0, 4.0])
    assert O.ldlt_solve(H, [2.0, 5.0, 8.0]).tolist() == [1.0, 0.0, 2.0] == R.ldlt_solve(H.tolist(), [2.0, 5.0, 8.0])


def test_oracle_converges_on_raycast_scans():
    from roborts_csm import worlds
    from roborts_csm.params import PARAM_CONFIG_OPTIMIZE, SIM_YAML_OPTIMIZE
    w = worlds.make_world(400, 400, 0.05, seed=3)
    b = worlds.make_scan_batch(w, 6, seed=5)
    m = O.Map(w.grid, w.resolution, w.offset)
    for prm in (SIM_YAML_OPTIMIZE, PARAM_CONFIG_OPTIMIZE):
        for k in range(6):
            pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
            c, p, it = O.optimize_scan_match(m, pts, prm, b.init_poses[k])
            d = p - b.true_poses[k]
            assert math.hypot(d[0], d[1]) < 0.03 and abs(d[2]) < 0.01, (k, d)
            assert c < 10.0 and 1 <= it <= prm.iterate_max_times


def test_oracle_early_returns(f1):
    from roborts_csm.params import SIM_YAML_OPTIMIZE
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]), update_index=-1)
    pose = np.array([0.1, 0.2, 0.3])
    c, p, _ = O.optimize_scan_match(m, f1["points"], SIM_YAML_OPTIMIZE, pose)
    assert c == 1000.0 and np.array_equal(p, pose)  # !IsMapInit (:73-76)
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    c, p, _ = O.optimize_scan_match(m, np.zeros((0, 2)), SIM_YAML_OPTIMIZE, pose)
    assert c == 1000.0 and np.array_equal(p, pose)  # empty scan


# ---------------------------------------------------------------- GPU parity
@pytest.fixture(scope="module")
def ctx():
    import roborts_csm
    c = roborts_csm.Context(0)
    yield c
    c.close()


def _set(ctx, grid, res, off, update_index=0):
    import roborts_csm
    ctx.set_grid(roborts_csm.ScanMatchMap(grid, float(res), tuple(off), update_index, 0), force=True)


@pytest.mark.gpu
def test_device_f6_bit_exact(ctx, f1, f6):
    _set(ctx, f1["grid"], f1["resolution"], f1["offset"])
    scans = _scans(f6)
    for tag in ("sim", "cfg"):
        prm = _prm(f6[f"param_{tag}"])
        poses = np.ascontiguousarray(f6["init_poses"], dtype=np.float64).copy()
        costs, iters = ctx.optimize_scan_match_batch(f6["points"], f6["offsets"], prm, poses)
        assert np.array_equal(costs, f6[f"cost_{tag}"]) and np.array_equal(poses, f6[f"pose_{tag}"]), tag
        assert np.array_equal(iters, f6[f"iters_{tag}"])
        for k, pts in enumerate(scans):  # single-scan entry point
            pose = np.array(f6["init_poses"][k], dtype=np.float64)
            c = ctx.optimize_scan_match(pts, prm, pose)
            assert c == f6[f"cost_{tag}"][k] and np.array_equal(pose, f6[f"pose_{tag}"][k]), (tag, k)


@pytest.mark.gpu
def test_device_batch_matches_oracle(ctx):
    """64 ray-cast scans on a 2000x2000 grid, and scans partly off the grid."""
    from roborts_csm import worlds
    from roborts_csm.params import PARAM_CONFIG_OPTIMIZE, SIM_YAML_OPTIMIZE, OptimizeScanMatchParam
    w = worlds.make_world(2000, 2000, 0.05, seed=11)
    b = worlds.make_scan_batch(w, 64, seed=12)
    _set(ctx, w.grid, w.resolution, w.offset)
    m = O.Map(w.grid, w.resolution, w.offset)
    init = b.init_poses.copy()
    init[5, :2] = [-w.offset[0] + 0.3, -w.offset[1] + 0.3]  # most endpoints off the map
    init[9, 2] += 1.5                                        # far off in angle
    for prm in (SIM_YAML_OPTIMIZE, PARAM_CONFIG_OPTIMIZE, OptimizeScanMatchParam(25, 0.0, 0.0, 0.05, 0.05),
                OptimizeScanMatchParam(0, 0.1, 0.5, 0.5, 0.5)):
        poses = np.ascontiguousarray(init).copy()
        costs, iters = ctx.optimize_scan_match_batch(b.points_cells, b.offsets, prm, poses)
        for k in range(64):
            pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
            c, p, it = O.optimize_scan_match(m, pts, prm, init[k])
            assert costs[k] == c and np.array_equal(poses[k], p) and iters[k] == it, (prm, k)


@pytest.mark.gpu
def test_device_early_returns(ctx, f1):
    from roborts_csm.params import SIM_YAML_OPTIMIZE
    pose = np.array([0.1, 0.2, 0.3])
    _set(ctx, f1["grid"], f1["resolution"], f1["offset"], update_index=-1)
    p = pose.copy()
    assert ctx.optimize_scan_match(f1["points"], SIM_YAML_OPTIMIZE, p) == 1000.0 and np.array_equal(p, pose)
    _set(ctx, f1["grid"], f1["resolution"], f1["offset"])
    p = pose.copy()
    assert ctx.optimize_scan_match(np.zeros((0, 2)), SIM_YAML_OPTIMIZE, p) == 1000.0 and np.array_equal(p, pose)
    # a mixed batch: empty scans between real ones
    pts = f1["points"]
    off = np.array([0, 0, len(pts), len(pts), 2 * len(pts)], dtype=np.int64)
    poses = np.tile(np.asarray(f1["init_pose"], dtype=np.float64), (4, 1))
    costs, _ = ctx.optimize_scan_match_batch(np.vstack([pts, pts]), off, SIM_YAML_OPTIMIZE, poses)
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    c, p, _ = O.optimize_scan_match(m, pts, SIM_YAML_OPTIMIZE, f1["init_pose"])
    assert costs.tolist() == [1000.0, c, 1000.0, c]
    assert np.array_equal(poses[1], p) and np.array_equal(poses[3], p)
    assert np.array_equal(poses[0], f1["init_pose"]) and np.array_equal(poses[2], f1["init_pose"])


def _oracle_scan_matchers(m, pts, levels, opt, failed, pose, cov, use_fine=True):
    """ScanMatchers::ScanMatch with use_optimize_scan_match (scan_matchers.h:189-288),
    composed from the oracle's two matchers (coarse map = fine map here)."""
    cost, proc, _ = O.optimize_scan_match(m, pts, opt, pose)
    score, times = failed / (cost + failed), 1
    if not use_fine or cost > failed:
        score, times, proc = 0.0, 0, np.array(pose, dtype=np.float64)
        r, proc, cov, _, _ = O.scan_match(m, pts, levels[0], proc, cov)
        score, times = score + r, times + 1
    if use_fine:
        for lv in levels[1:]:
            r, proc, cov, _, _ = O.scan_match(m, pts, lv, proc, cov)
            score, times = score + r, times + 1
    return score / times, proc, cov


@pytest.mark.gpu
@pytest.mark.parametrize("failed", [2.0, 0.5, 0.05])
def test_device_scan_matchers_with_optimizer(ctx, failed):
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.params import SIM_YAML_LEVELS, SIM_YAML_OPTIMIZE
    w = worlds.make_world(600, 600, 0.05, seed=21)
    b = worlds.make_scan_batch(w, 6, seed=22)
    smap = roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 1)
    m = O.Map(w.grid, w.resolution, w.offset)
    sm = roborts_csm.ScanMatchers(SIM_YAML_LEVELS, ctx, use_optimize_scan_match=True,
                                  optimize=SIM_YAML_OPTIMIZE, optimize_failed_cost=failed)
    for k in range(6):
        pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
        rd = roborts_csm.RangeDataContainer2d(pts)
        for use_fine in (True, False):
            pose = np.array(b.init_poses[k], dtype=np.float64)
            cov = np.eye(3)
            s = sm.ScanMatch(rd, rd, smap, smap, pose, cov, use_fine)
            s2, p2, c2 = _oracle_scan_matchers(m, pts, SIM_YAML_LEVELS, SIM_YAML_OPTIMIZE, failed,
                                               b.init_poses[k], np.eye(3), use_fine)
            assert s == s2 and np.array_equal(pose, p2) and np.array_equal(cov.reshape(-1), c2), (k, use_fine)


def test_sincos_is_not_cos_and_sin():
    """The trap host_math.hpp / oracle_math.hpp guard against: glibc's sincos
    and separate cos/sin disagree in the last bit for some arguments, so the
    restatements must pick the one the reference's GCC build calls (sincos)."""
    from libm import sincos
    rng = np.random.default_rng(0)
    xs = rng.uniform(-4, 4, 20000)
    diff = sum((sincos(x) != (math.cos(x), math.sin(x))) for x in xs)
    assert diff > 0  # if glibc ever makes them agree, the guard is merely redundant


@pytest.mark.gpu
def test_device_update_cost_matches_oracle(ctx):
    """One UpdateCost on the device at 200 random map-cell poses (test hook)."""
    from roborts_csm import worlds
    w = worlds.make_world(800, 800, 0.05, seed=31)
    b = worlds.make_scan_batch(w, 10, seed=32)
    _set(ctx, w.grid, w.resolution, w.offset)
    m = O.Map(w.grid, w.resolution, w.offset)
    rng = np.random.default_rng(33)
    for k in range(10):
        pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
        e0 = O.world_to_map(m, b.init_poses[k])
        for _ in range(20):
            e = e0 + rng.normal(size=3) * [3.0, 3.0, 0.1]
            c1, H1, b1 = ctx.optimize_update_cost(pts, e)
            c2, H2, b2 = O.optimize_update_cost(m, pts, e)
            assert c1 == c2 and np.array_equal(H1, H2) and np.array_equal(b1, b2)
