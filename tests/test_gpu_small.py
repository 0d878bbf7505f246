"""The few-window path (csm_split.hip, the 16-wave fast finish, FinishOut and
a done flag written straight into pinned host memory): the reference's own
calling pattern, one scan at a time through ScanMatchers::ScanMatch
(scan_matchers.h:238-256), at the map resolutions it ships.

  1 cm fine map (config/simulatin_param.yaml:28,51-70): window steps of
      5, 2 and 1 cells; ParamConfig defaults (param_config.h:71-90): 10, 2, 1
  2.5 cm real-robot map (config/real_robot_param.yaml): 2, 0.8 and 0.4 cells

Every score, the argmax, pose, covariance and response are compared with the
oracle bit for bit (tolerance 0), and the split kernel is checked to be the
one that ran.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import pyoracle as O  # noqa: E402


def _ctx(**env):
    import roborts_csm
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return roborts_csm.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def ctx():
    c = _ctx()
    yield c
    c.close()


def _map(w):
    import roborts_csm
    return roborts_csm.ScanMatchMap(w.grid, float(w.resolution), tuple(w.offset), 0, 1)


@pytest.fixture(scope="module")
def world1cm():
    from roborts_csm import worlds
    w = worlds.make_world(1200, 1200, 0.01, seed=31)
    return w, worlds.make_scan_batch(w, 12, seed=5)


@pytest.fixture(scope="module")
def world25():
    from roborts_csm import worlds
    w = worlds.make_world(800, 800, 0.025, seed=32)
    return w, worlds.make_scan_batch(w, 12, seed=6)


def _levels(name):
    from roborts_csm.params import PARAM_CONFIG_LEVELS, SIM_YAML_LEVELS, headline_levels
    return {"sim": SIM_YAML_LEVELS, "pcfg": PARAM_CONFIG_LEVELS, "b1081": headline_levels()}[name]


def _steps(levels, res):
    return [l.search_space_resolution / (1 / (1 / res)) for l in levels]


@pytest.mark.parametrize("wname,lname,want_steps", [
    ("world1cm", "sim", [5.0, 2.0, 1.0]),
    ("world1cm", "pcfg", [10.0, 2.0, 1.0]),
    ("world1cm", "b1081", [5.0, 2.0, 1.0]),
    ("world25", "sim", [2.0, 0.8, 0.4]),
])
def test_split_scores_bit_exact(ctx, request, wname, lname, want_steps):
    """All scores of each level's window, single scans, against the oracle."""
    w, b = request.getfixturevalue(wname)
    levels = _levels(lname)
    assert np.allclose(_steps(levels, w.resolution), want_steps)
    ctx.set_grid(_map(w))
    m = O.Map(w.grid, w.resolution, w.offset)
    ctx.set_profiling(True)
    for k in range(3):
        pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
        c = O.world_to_map(m, b.init_poses[k])
        for lv in levels:
            got = ctx.score_window(pts, lv, c)
            want = O.score_window(m, pts, lv, c, got.size)
            assert np.array_equal(got, want), (wname, lname, lv)
    names = {s["name"] for s in ctx.kernel_stats()}
    ctx.set_profiling(False)
    assert any(n.startswith("score_split_kernel") for n in names), names


@pytest.mark.parametrize("wname,lname", [("world1cm", "sim"), ("world1cm", "pcfg"), ("world1cm", "b1081"),
                                         ("world25", "sim"), ("world25", "b1081")])
def test_split_three_levels_bit_exact(ctx, request, wname, lname):
    """ScanMatchers::ScanMatch per scan: response, pose and covariance."""
    w, b = request.getfixturevalue(wname)
    levels = _levels(lname)
    ctx.set_grid(_map(w))
    m = O.Map(w.grid, w.resolution, w.offset)
    for k in range(b.offsets.size - 1):
        pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
        pose = np.array(b.init_poses[k], dtype=np.float64)
        cov = np.eye(3).reshape(9).copy()
        s = ctx.scan_matchers(pts, levels, pose, cov)
        s2, p2, c2 = O.scan_matchers(m, pts, levels, b.init_poses[k], np.eye(3))
        assert s == s2 and np.array_equal(pose, p2) and np.array_equal(cov, c2), (k, s, s2, pose, p2)


@pytest.mark.parametrize("n", [1, 2, 7, 32])
def test_split_batches_bit_exact(ctx, world1cm, n):
    """Windows per launch 1..32 (the split path's range): each scan's
    response, argmax, pose and covariance equal the oracle's single call."""
    from roborts_csm.params import SIM_YAML_LEVELS
    w, b = world1cm
    ctx.set_grid(_map(w))
    m = O.Map(w.grid, w.resolution, w.offset)
    idx = [k % (b.offsets.size - 1) for k in range(n)]
    pts = np.concatenate([b.points_cells[b.offsets[k]:b.offsets[k + 1]] for k in idx])
    off = np.zeros(n + 1, dtype=np.int64)
    off[1:] = np.cumsum([b.offsets[k + 1] - b.offsets[k] for k in idx])
    # distinct centres per window
    init = np.array([b.init_poses[k] + [0.003 * j, -0.002 * j, 0.001 * j] for j, k in enumerate(idx)])
    for lv in SIM_YAML_LEVELS:
        poses = np.ascontiguousarray(init.copy())
        covs = np.tile(np.eye(3).reshape(1, 9), (n, 1))
        r, am = ctx.scan_match_batch(pts, off, lv, poses, covs)
        for j in range(n):
            p = pts[off[j]:off[j + 1]]
            r2, p2, c2, am2, _ = O.scan_match(m, p, lv, init[j], np.eye(3))
            assert r[j] == r2 and am[j] == am2 and np.array_equal(poses[j], p2), j
            assert np.array_equal(covs[j], c2), j


def test_split_matches_throughput_kernels(world1cm, world25):
    """CSM_SMALL=0 (the throughput kernels: column / phase / tiny / box) and
    the split path agree on every output for single scans."""
    from roborts_csm.params import PARAM_CONFIG_LEVELS, SIM_YAML_LEVELS
    a, b_ = _ctx(), _ctx(CSM_SMALL=0)
    try:
        for w, b in (world1cm, world25):
            for c in (a, b_):
                c.set_grid(_map(w))
            for levels in (SIM_YAML_LEVELS, PARAM_CONFIG_LEVELS):
                for k in range(4):
                    pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
                    out = []
                    for c in (a, b_):
                        pose = np.array(b.init_poses[k], dtype=np.float64)
                        cov = np.eye(3).reshape(9).copy()
                        s = c.scan_matchers(pts, levels, pose, cov)
                        out.append((s, pose, cov))
                    assert out[0][0] == out[1][0]
                    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])
    finally:
        a.close()
        b_.close()


def test_split_windows_off_the_grid(ctx, world1cm):
    """Windows hanging off every edge (negative and past-the-end indices read
    `outside`), with and without the centre penalty."""
    from roborts_csm.params import SIM_YAML_LEVELS
    w, b = world1cm
    ctx.set_grid(_map(w))
    m = O.Map(w.grid, w.resolution, w.offset)
    pts = b.points_cells[b.offsets[0]:b.offsets[1]]
    for cx, cy in ((-3.0, 5.0), (5.0, -40.0), (w.size_x + 2.0, 600.0), (600.0, w.size_y - 1.0), (-500.0, -500.0)):
        for lv in SIM_YAML_LEVELS:
            for pen in (True, False):
                p = lv.with_(use_center_penalty=pen)
                c = np.array([cx, cy, 0.3])
                got = ctx.score_window(pts, p, c)
                assert np.array_equal(got, O.score_window(m, pts, p, c, got.size)), (cx, cy, lv)


def test_split_many_splits_and_few_beams(ctx, world1cm):
    """Beam counts around the split boundaries (1, 31, 32, 33, 64, 1081 beams:
    1 to 34 splits of at most 32 beams), every score against the oracle."""
    from roborts_csm.params import SIM_YAML_LEVELS
    w, b = world1cm
    ctx.set_grid(_map(w))
    m = O.Map(w.grid, w.resolution, w.offset)
    full = b.points_cells[b.offsets[1]:b.offsets[2]]
    c = O.world_to_map(m, b.init_poses[1])
    for n in (1, 31, 32, 33, 64, min(1081, full.shape[0])):
        pts = full[:n]
        for lv in SIM_YAML_LEVELS:
            p = lv.with_(use_point_size=2000)  # every beam summed
            got = ctx.score_window(pts, p, c)
            assert np.array_equal(got, O.score_window(m, pts, p, c, got.size)), (n, lv)
