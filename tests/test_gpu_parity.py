"""GPU parity: the HIP path (through the C-ABI of libroborts_csm.so) against
the CPU oracle and the committed golden fixtures.

Bar (north star): bit-exact argmax pose index, scores within 1e-6 — this
implementation is held to bit-exact everywhere (scores, sort order, pose,
covariance, response), tolerance 0.
"""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import pyoracle as O  # noqa: E402


def _param(a):
    from roborts_csm.params import CorrelationScanMatchParam
    return CorrelationScanMatchParam(float(a[0]), float(a[1]), float(a[2]), float(a[3]), float(a[4]),
                                     int(a[5]), int(a[6]), bool(a[7]), int(a[8]))


@pytest.fixture(scope="module")
def ctx():
    import roborts_csm
    c = roborts_csm.Context(0)
    yield c
    c.close()


def _map(grid, res, off, update_index=0, version=0):
    import roborts_csm
    return roborts_csm.ScanMatchMap(grid, float(res), tuple(off), update_index, version)


def _variant_ctx(kern, **env):
    """A context of one kernel family. kern: a CSM_KERNEL value, None for the
    default throughput kernels (box / phase / tiny), "split" for the
    few-window path (tests/test_gpu_small.py), which single-window calls take
    by default; every other variant turns it off (CSM_SMALL=0)."""
    import roborts_csm
    env = dict(env)
    if kern != "split":
        env["CSM_SMALL"] = "0"
        if kern:
            env["CSM_KERNEL"] = kern
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return roborts_csm.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def f1(golden_dir):
    return np.load(os.path.join(golden_dir, "f1_config1.npz"))


def test_f1_scores_bit_exact(ctx, f1):
    ctx.set_grid(_map(f1["grid"], f1["resolution"], f1["offset"]), force=True)
    sc = ctx.score_window(f1["points"], _param(f1["param"]), f1["center"])
    assert sc.size == 7056
    assert np.array_equal(sc, f1["scores"])


def test_f1_scan_match_bit_exact(ctx, f1):
    ctx.set_grid(_map(f1["grid"], f1["resolution"], f1["offset"]), force=True)
    pose = np.array(f1["init_pose"], dtype=np.float64)
    cov = np.eye(3).reshape(9).copy()
    r, am = ctx.scan_match(f1["points"], _param(f1["param"]), pose, cov, return_argmax=True)
    assert am == f1["argmax"]
    assert r == f1["response"]
    assert np.array_equal(pose, f1["pose"]) and np.array_equal(cov, f1["cov"])


def test_f1_three_level_bit_exact(ctx, f1):
    from roborts_csm.params import SIM_YAML_LEVELS
    ctx.set_grid(_map(f1["grid"], f1["resolution"], f1["offset"]), force=True)
    pose = np.array(f1["init_pose"], dtype=np.float64)
    cov = np.eye(3).reshape(9).copy()
    s = ctx.scan_matchers(f1["points"], SIM_YAML_LEVELS, pose, cov)
    assert s == f1["sim3_score"]
    assert np.array_equal(pose, f1["sim3_pose"]) and np.array_equal(cov, f1["sim3_cov"])


@pytest.mark.parametrize("tag", ["sim", "b1081", "pcfg"])
def test_f2_levels_bit_exact(ctx, golden_dir, tag):
    f2 = np.load(os.path.join(golden_dir, "f2_config2_crop.npz"))
    ctx.set_grid(_map(f2["grid"], f2["resolution"], f2["offset"]), force=True)
    levels = [_param(a) for a in f2[f"{tag}_levels"]]
    for li in range(3):
        sc = ctx.score_window(f2["points"], levels[li], f2[f"{tag}_l{li}_center"])
        assert np.array_equal(sc, f2[f"{tag}_l{li}_scores"]), (tag, li)
    pose = np.array(f2["init_pose"], dtype=np.float64)
    cov = np.eye(3).reshape(9).copy()
    s = ctx.scan_matchers(f2["points"], levels, pose, cov)
    assert s == f2[f"{tag}_score"]
    assert np.array_equal(pose, f2[f"{tag}_pose"]) and np.array_equal(cov, f2[f"{tag}_cov"])


def test_f3_ties_bit_exact(ctx, golden_dir):
    """Whole groups of candidates tie: the winner depends on std::sort's order."""
    f3 = np.load(os.path.join(golden_dir, "f3_ties.npz"))
    ctx.set_grid(_map(f3["grid"], f3["resolution"], f3["offset"]), force=True)
    for tag in ("pen", "nopen", "fine"):
        p = _param(f3[f"{tag}_param"])
        pose = np.array(f3["init_pose"], dtype=np.float64)
        cov = np.eye(3).reshape(9).copy()
        r, am = ctx.scan_match(f3["points"], p, pose, cov, return_argmax=True)
        assert am == f3[f"{tag}_argmax"], tag
        assert r == f3[f"{tag}_response"]
        assert np.array_equal(pose, f3[f"{tag}_pose"]) and np.array_equal(cov, f3[f"{tag}_cov"])


def test_f5_best_window(ctx, golden_dir, f1):
    f5 = np.load(os.path.join(golden_dir, "f5_large_window.npz"))
    ctx.set_grid(_map(f1["grid"], f1["resolution"], f1["offset"]), force=True)
    b = ctx.best_window(f1["points"], _param(f5["param"]), f5["center"])
    assert b.score == f5["best_score"] and b.flat_index == f5["best_flat"]


def test_hostile_grid_bit_exact(ctx, f1):
    """fp32 values over 30 binades: fp64 sums are order-dependent here, so
    only the reference beam order reproduces the oracle bit for bit."""
    from roborts_csm import worlds
    g = worlds.hostile_grid(400, 400)
    ctx.set_grid(_map(g, f1["resolution"], f1["offset"]), force=True)
    m = O.Map(g, float(f1["resolution"]), tuple(f1["offset"]))
    p = _param(f1["param"])
    for U in (100, 1000):
        q = p.with_(use_point_size=U)
        sc = ctx.score_window(f1["points"], q, f1["center"])
        ref = O.score_window(m, f1["points"], q, f1["center"], sc.size)
        assert np.array_equal(sc, ref)


def test_aos_cells_upload(ctx, f1):
    g = f1["grid"]
    aos = np.zeros(g.shape, dtype=[("prob_value_", "<f4"), ("update_index_", "<i4")])
    aos["prob_value_"] = g
    aos["update_index_"] = 7
    ctx.set_grid(_map(aos, f1["resolution"], f1["offset"]), force=True)
    sc = ctx.score_window(f1["points"], _param(f1["param"]), f1["center"])
    assert np.array_equal(sc, f1["scores"])


def test_out_of_bounds_endpoints(ctx):
    """Endpoints beyond the grid read the defined outside value (the reference
    reads out of bounds: UB). Both sides use the same definition."""
    rng = np.random.default_rng(5)
    g = rng.uniform(0.3, 1.0, size=(64, 80)).astype(np.float32)
    pts = rng.uniform(-120, 120, size=(500, 2))
    from roborts_csm.params import CONFIG1_PARAM
    p = CONFIG1_PARAM.with_(use_point_size=400)
    center = np.array([40.0, 30.0, 0.2])
    ctx.set_grid(_map(g, 0.05, (0.0, 0.0)), force=True)
    for outside in (0.3, 0.0, 0.75):
        ctx.set_outside_value(outside)
        m = O.Map(g, 0.05, (0.0, 0.0), outside=outside)
        sc = ctx.score_window(pts, p, center)
        assert np.array_equal(sc, O.score_window(m, pts, p, center, sc.size))
    ctx.set_outside_value(0.3)


@pytest.mark.parametrize("n,U", [(1, 100), (1, 1), (150, 100), (199, 100), (200, 100), (1081, 541),
                                 (1081, 540), (1081, 1081), (3000, 5000), (5000, 2)])
def test_beam_subsampling_edges(ctx, f1, n, U):
    """The :561-566 rule (step, divisor) at its boundaries, incl. >1 LDS chunk."""
    rng = np.random.default_rng(n * 7 + U)
    pts = rng.uniform(-60, 60, size=(n, 2))
    p = _param(f1["param"]).with_(use_point_size=U)
    ctx.set_grid(_map(f1["grid"], f1["resolution"], f1["offset"]), force=True)
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    sc = ctx.score_window(pts, p, f1["center"])
    assert np.array_equal(sc, O.score_window(m, pts, p, f1["center"], sc.size))
    pose = np.array(f1["init_pose"], dtype=np.float64)
    cov = np.eye(3).reshape(9).copy()
    r, am = ctx.scan_match(pts, p, pose, cov, return_argmax=True)
    r2, pose2, cov2, am2, _ = O.scan_match(m, pts, p, f1["init_pose"], np.eye(3))
    assert (r, am) == (r2, am2)
    assert np.array_equal(pose, pose2) and np.array_equal(cov, cov2)


def test_early_returns(ctx, f1):
    """Uninitialised map or empty scan: response 0, pose/cov untouched (:792-795)."""
    p = _param(f1["param"])
    ctx.set_grid(_map(f1["grid"], f1["resolution"], f1["offset"], update_index=-1), force=True)
    pose = np.array(f1["init_pose"], dtype=np.float64)
    cov = np.full(9, 7.0)
    r, am = ctx.scan_match(f1["points"], p, pose, cov, return_argmax=True)
    assert r == 0.0 and am == -1 and np.array_equal(pose, f1["init_pose"]) and (cov == 7.0).all()
    ctx.set_grid(_map(f1["grid"], f1["resolution"], f1["offset"]), force=True)
    r = ctx.scan_match(np.zeros((0, 2)), p, pose, cov)
    assert r == 0.0 and np.array_equal(pose, f1["init_pose"]) and (cov == 7.0).all()


def test_invalid_use_point_size(ctx, f1):
    import roborts_csm
    ctx.set_grid(_map(f1["grid"], f1["resolution"], f1["offset"]), force=True)
    p = _param(f1["param"]).with_(use_point_size=1)
    with pytest.raises(roborts_csm.CsmError) as e:
        ctx.scan_match(f1["points"], p, np.array(f1["init_pose"], dtype=np.float64), np.eye(3).reshape(9).copy())
    assert e.value.status == 1


def test_grid_version_cache(ctx, f1):
    g = np.array(f1["grid"])
    p = _param(f1["param"])
    m = _map(g, f1["resolution"], f1["offset"], version=11)
    ctx.set_grid(m)
    a = ctx.score_window(f1["points"], p, f1["center"])
    g[:, :] = np.float32(0.5)          # same buffer, same version -> cached copy is used
    ctx.set_grid(m)
    assert np.array_equal(ctx.score_window(f1["points"], p, f1["center"]), a)
    m.version = 12                     # bump -> re-upload
    ctx.set_grid(m)
    b = ctx.score_window(f1["points"], p, f1["center"])
    assert not np.array_equal(a, b)


@pytest.fixture(scope="module")
def world2000():
    from roborts_csm import worlds
    w = worlds.make_world(2000, 2000, 0.05)
    b = worlds.make_scan_batch(w, 96, seed=99)
    return w, b


@pytest.mark.parametrize("which", ["sim", "headline"])
def test_batch_three_level_bit_exact(ctx, world2000, which):
    """BASELINE config 2 shape (1081 beams, 2000x2000 @5 cm), batched 3 levels."""
    from roborts_csm.params import SIM_YAML_LEVELS, headline_levels
    w, b = world2000
    levels = SIM_YAML_LEVELS if which == "sim" else headline_levels()
    ctx.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
    poses = np.ascontiguousarray(b.init_poses.copy())
    covs = np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1))
    s = ctx.scan_matchers_batch(b.points_cells, b.offsets, levels, poses, covs)
    m = O.Map(w.grid, w.resolution, w.offset)
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, levels, b.init_poses,
                                       np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1)))
    assert np.array_equal(s, s2)
    assert np.array_equal(poses, p2)
    assert np.array_equal(covs, c2)
    # property: the matcher pulls the (0.12, -0.07, 4 deg) init error in
    err = np.hypot(*(poses[:, :2] - b.true_poses[:, :2]).T)
    assert np.median(err) < 0.05


def test_headline_runs_row_segment_kernels(ctx, world2000):
    """The config-2 levels run on the box kernel (coarse: one-cell step), the
    phase kernel (fine: 0.4-cell step) and the tiny-window kernel (super-fine:
    a 0.4-cell span), not a fallback, and the device finish, and the result is
    the oracle's bit for bit."""
    from roborts_csm.params import headline_levels
    w, b = world2000
    ctx.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
    n = 48  # above the few-window path's 32 (tests/test_gpu_small.py)
    poses = np.ascontiguousarray(b.init_poses[:n].copy())
    covs = np.tile(np.eye(3).reshape(1, 9), (n, 1))
    ctx.set_profiling(True)
    s = ctx.scan_matchers_batch(b.points_cells[:b.offsets[n]], b.offsets[:n + 1], headline_levels(), poses, covs)
    names = {k["name"] for k in ctx.kernel_stats()}
    ctx.set_profiling(False)
    for want in ("score_box_pair_kernel<13,all>", "score_phase_kernel<11,all>",
                 "score_tiny_kernel<3,all>", "finish_kernel<5070>"):
        assert want in names, names
    m = O.Map(w.grid, w.resolution, w.offset)
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells[:b.offsets[n]], b.offsets[:n + 1], headline_levels(),
                                       b.init_poses[:n], np.tile(np.eye(3).reshape(1, 9), (n, 1)))
    assert np.array_equal(s, s2) and np.array_equal(poses, p2) and np.array_equal(covs, c2)


def test_batch_single_level_matches_single_calls(ctx, world2000):
    from roborts_csm.params import SIM_YAML_LEVELS
    w, b = world2000
    ctx.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
    n = 16
    poses = np.ascontiguousarray(b.init_poses[:n].copy())
    covs = np.tile(np.eye(3).reshape(1, 9), (n, 1))
    r, am = ctx.scan_match_batch(b.points_cells[:b.offsets[n]], b.offsets[:n + 1], SIM_YAML_LEVELS[0], poses, covs)
    for k in range(n):
        pose = np.array(b.init_poses[k])
        cov = np.eye(3).reshape(9).copy()
        r1, am1 = ctx.scan_match(b.points_cells[b.offsets[k]:b.offsets[k + 1]], SIM_YAML_LEVELS[0], pose, cov,
                                 return_argmax=True)
        assert r1 == r[k] and am1 == am[k]
        assert np.array_equal(pose, poses[k]) and np.array_equal(cov, covs[k])


def test_best_window_large_matches_oracle(ctx, world2000):
    """Argmax-only over a +-2 m / +-180 deg window at full grid size."""
    from roborts_csm.params import CorrelationScanMatchParam
    w, b = world2000
    ctx.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
    p = CorrelationScanMatchParam(2.0, 0.05, math.pi, 0.0349, 0.5, 100, 0, False, 0)
    m = O.Map(w.grid, w.resolution, w.offset)
    for k in range(3):
        pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
        c = O.world_to_map(m, b.init_poses[k])
        got = ctx.best_window(pts, p, c)
        s, flat = O.best_window(m, pts, p, c)
        assert got.score == s and got.flat_index == flat


@pytest.mark.parametrize("levels", ["sim", "headline"])
def test_device_finish_equals_host_sort(world2000, levels):
    """CSM_FINISH=host (std::sort on the host), CSM_FINISH=exact (the device
    std::sort emulation on every window) and the default device finish (the
    fast no-sort path, exact emulation only where ties matter) give identical
    poses, covariances, scores and argmax indices; the fast path is taken."""
    import roborts_csm
    from roborts_csm.params import SIM_YAML_LEVELS, headline_levels
    w, b = world2000
    ctxs = []
    for mode in ("host", "exact", None):
        if mode:
            os.environ["CSM_FINISH"] = mode
        try:
            ctxs.append(roborts_csm.Context(0))
        finally:
            os.environ.pop("CSM_FINISH", None)
    lvs = SIM_YAML_LEVELS if levels == "sim" else headline_levels()
    out = []
    for c in ctxs:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
        c.set_profiling(True)
        res = []
        for lv in lvs:
            poses = np.ascontiguousarray(b.init_poses.copy())
            covs = np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1))
            r, am = c.scan_match_batch(b.points_cells, b.offsets, lv, poses, covs)
            res.append((r, am, poses, covs))
        out.append(res)
    st = {k["name"]: k for k in ctxs[2].kernel_stats()}
    for c in ctxs:
        c.close()
    for other in out[1:]:
        for a, d in zip(out[0], other):
            for x, y in zip(a, d):
                assert np.array_equal(x, y)
    # most windows settled without the sort
    assert st["finish:exact_windows"]["scorings"] < 0.5 * 3 * b.offsets.size


def test_device_finish_ties_random_windows(ctx):
    """Tie-heavy windows (coarse grid values on a sub-cell window step) through
    the device sort, against the oracle's std::sort."""
    from roborts_csm.params import SIM_YAML_LEVELS
    rng = np.random.default_rng(17)
    g = rng.choice(np.array([0.3, 0.5, 0.7, 1.0], dtype=np.float32), size=(300, 300))
    ctx.set_grid(_map(g, 0.05, (7.5, 7.5)), force=True)
    m = O.Map(g, 0.05, (7.5, 7.5))
    for t in range(12):
        pts = rng.uniform(-80, 80, size=(int(rng.integers(20, 400)), 2))
        init = rng.uniform(-1, 1, size=3)
        for lv in SIM_YAML_LEVELS:
            lv = lv.with_(use_center_penalty=bool(t % 2))
            pose = init.copy()
            cov = np.eye(3).reshape(9).copy()
            r, am = ctx.scan_match(pts, lv, pose, cov, return_argmax=True)
            r2, pose2, cov2, am2, _ = O.scan_match(m, pts, lv, init, np.eye(3))
            assert (r, am) == (r2, am2), (t, lv)
            assert np.array_equal(pose, pose2) and np.array_equal(cov, cov2)


@pytest.mark.parametrize("grid_kind", ["blur", "hostile", "coarse_values"])
def test_kernel_variants_agree(f1, grid_kind):
    """v1 (lane per candidate, fp64), v2 fp64 and v2 fixed-point column
    kernels all reproduce the oracle bit for bit (which one runs depends on
    the grid: the fixed-point path needs exactly summable cell values)."""
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.params import PARAM_CONFIG_LEVELS, SIM_YAML_LEVELS
    rng = np.random.default_rng(23)
    if grid_kind == "blur":
        g = f1["grid"]
    elif grid_kind == "hostile":
        g = worlds.hostile_grid(400, 400)
    else:
        g = rng.choice(np.array([0.3, 0.41, 0.88, 1.0], dtype=np.float32), size=(400, 400))
    m = O.Map(g, float(f1["resolution"]), tuple(f1["offset"]))
    # None: default throughput kernels (v11 pair box / v7 phase over strips / v8 tiny / v4); split:
    # few-window path; the last: v6 box and the phase kernel over gridi
    ctxs = [_variant_ctx(k) for k in ("v2", "v4", "v6", "v7", None, "split")]
    ctxs.append(_variant_ctx("v8", CSM_PHASE_STRIPS="0"))
    params = [_param(f1["param"])] + list(SIM_YAML_LEVELS) + [l.with_(use_point_size=1081) for l in SIM_YAML_LEVELS]
    params += [l.with_(use_point_size=1081) for l in PARAM_CONFIG_LEVELS]
    for c in ctxs:
        c.set_grid(_map(g, f1["resolution"], f1["offset"]), force=True)
        for p in params:
            sc = c.score_window(f1["points"], p, f1["center"])
            assert np.array_equal(sc, O.score_window(m, f1["points"], p, f1["center"], sc.size)), (grid_kind, p)
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("thin", [1, 10])
def test_box_kernel_edge_beams(world2000, thin):
    """v6 box kernel (one-cell window step) on its margin cases: beams whose
    (lx + x0) + 0.5 is an exact integer (points at the origin, window with
    x0 + 0.5 integral), beams off the grid's low edge (negative t, where the
    reference's truncation is not a floor) and past its high edges, and windows
    whose x0 + j crosses a power of two (inexact steps) -- all scores and the
    argmax against the oracle and against the v4 row kernel. thin = 10: every
    10th beam plus the edge beams, 116 in all, the pair kernel's run-free
    short-scan form (kPairNoRunBeams)."""
    import roborts_csm
    from roborts_csm.params import SIM_YAML_LEVELS
    w, b = world2000
    m = O.Map(w.grid, w.resolution, w.offset)
    pts = b.points_cells[b.offsets[0]:b.offsets[1]][::thin]
    extra = np.array([[0.0, 0.0], [0.0, 0.0], [1.0, -2.0], [-1500.0, 3.0], [2.0, -1500.0],
                      [900.0, 900.0], [-3000.0, -3000.0], [0.25, 0.0]])
    pts = np.ascontiguousarray(np.concatenate([pts, extra]))
    lv = SIM_YAML_LEVELS[0].with_(use_point_size=pts.shape[0])
    half = (lv.search_space_size / w.resolution) * 0.5
    c0 = 100.5 + half
    assert float(c0 - half) + 0.5 == 101.0  # origin points sit exactly on a rounding boundary
    centers = [[c0, 200.5 + half, 0.0], [c0, 200.5 + half, 1.3],
               [1020.0 + 3 * 2.0 ** -43, 1019.0 + 2.0 ** -43, 0.7],
               [6.2, 3.1, -2.5], [1995.0, 1990.0, 1.0], [511.0 + 2.0 ** -44, 250.3, 3.0]]
    # None: the v11 pair box kernel (the world's 7 values); v8: the v6 box kernel over gridi
    ctxs = [_variant_ctx(k) for k in (None, "v4", "split", "v8")]
    for c in ctxs:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
    for i in (0, 3):
        ctxs[i].set_profiling(True)
    for cen in centers:
        cen = np.array(cen)
        want = O.score_window(m, pts, lv, cen, 30 * 13 * 13)
        for c in ctxs:
            assert np.array_equal(c.score_window(pts, lv, cen), want), cen
            got = c.best_window(pts, lv, cen)
            s, flat = O.best_window(m, pts, lv, cen)
            assert got.score == s and got.flat_index == flat
    for i, kn in ((0, "score_box_pair_kernel"), (3, "score_box_kernel")):
        names = {k["name"] for k in ctxs[i].kernel_stats()}
        assert kn + "<13,all>" in names and kn + "<13,best>" in names, (i, names)
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("size,penalty", [(0.8, True), (0.85, False), (1.55, True), (1.6, False), (3.0, True)])
def test_box_tiles_large_windows(world2000, size, penalty):
    """One-cell-step windows wider than 16 (loop closure): the box kernel over
    16 x 16 tiles (the last one shifted back to the edge) against the column
    kernel (CSM_KERNEL=v2) and the oracle: score and flat index bit for bit,
    with beams on rounding boundaries (the cell-by-cell path at tile offsets),
    windows hanging off the grid and the centre penalty on and off."""
    import roborts_csm
    from roborts_csm.params import CorrelationScanMatchParam
    w, b = world2000
    m = O.Map(w.grid, w.resolution, w.offset)
    pts = b.points_cells[b.offsets[1]:b.offsets[2]]
    extra = np.array([[0.0, 0.0], [0.0, 0.0], [1.0, -2.0], [-1500.0, 3.0], [900.0, 900.0], [0.25, 0.0]])
    pts = np.ascontiguousarray(np.concatenate([pts, extra]))
    p = CorrelationScanMatchParam(size, 0.05, 0.3, 0.0349, 0.5, pts.shape[0], 0, penalty, 0)
    na, ns = roborts_csm.window_dims(p)
    assert ns > 16
    half = (size / w.resolution) * 0.5
    assert float(100.5 + half - half) + 0.5 == 101.0  # origin points on a rounding boundary
    centers = [[100.5 + half, 200.5 + half, 0.0], [1020.0 + 3 * 2.0 ** -43, 1019.0 + 2.0 ** -43, 0.7],
               [6.2, 3.1, -2.5], [1995.0, 1990.0, 1.0]]
    ctxs = []
    for kern in (None, "v2"):
        if kern:
            os.environ["CSM_KERNEL"] = kern
        try:
            ctxs.append(roborts_csm.Context(0))
        finally:
            os.environ.pop("CSM_KERNEL", None)
    try:
        for c in ctxs:
            c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
        ctxs[0].set_profiling(True)
        cen = np.array(centers)
        got = [c.best_windows(pts, p, np.zeros(len(centers), dtype=np.int32), cen) for c in ctxs]
        for i in range(len(centers)):
            s, flat = O.best_window(m, pts, p, cen[i])
            for g in got:
                assert g[0][i] == s and g[1][i] == flat, (i, g[0][i], s, g[1][i], flat)
        names = {k["name"] for k in ctxs[0].kernel_stats()}
        assert "score_box_kernel<16,best,tiles>" in names, names
        assert not any(n.startswith("score_box_kernel") for n in {k["name"] for k in ctxs[1].kernel_stats()})
    finally:
        for c in ctxs:
            c.close()


def test_fixed_point_path_out_of_grid(ctx):
    """Exactly-summable grid (the fixed-point kernel) with endpoints far
    outside it: the hardware range check must read the outside value."""
    rng = np.random.default_rng(29)
    g = rng.choice(np.array([0.3, 0.5, 0.7, 1.0], dtype=np.float32), size=(50, 70))
    pts = rng.uniform(-400, 400, size=(700, 2))
    from roborts_csm.params import SIM_YAML_LEVELS
    ctx.set_grid(_map(g, 0.05, (0.0, 0.0)), force=True)
    for outside in (0.3, 0.0, 0.5):
        ctx.set_outside_value(outside)
        m = O.Map(g, 0.05, (0.0, 0.0), outside=outside)
        for lv in SIM_YAML_LEVELS:
            for center in ([25.0, 35.0, 0.3], [-30.0, 90.0, 2.0], [69.6, 0.2, -1.0]):
                p = lv.with_(use_point_size=700)
                sc = ctx.score_window(pts, p, np.array(center))
                assert np.array_equal(sc, O.score_window(m, pts, p, np.array(center), sc.size))
    ctx.set_outside_value(0.3)


def _killer(n):
    """Median-of-3 killer-ish sequences that drive introsort to its depth limit."""
    k = np.zeros(n)
    half = n // 2
    for i in range(half):
        k[2 * i] = i + 1
        k[2 * i + 1] = half + i + 1
    return k[::-1].copy()


@pytest.mark.parametrize("seed", [0, 1])
def test_device_sort_matches_libstdcxx(ctx, seed):
    """The finish kernel's sort == libstdc++ std::sort(greater), ties and
    depth-limit heap sort included."""
    rng = np.random.default_rng(seed)
    cases = [np.zeros(5070), np.ones(17), (np.arange(5070) % 2).astype(float), _killer(4096),
             _killer(5070), np.arange(10240, dtype=float), np.arange(10240, dtype=float)[::-1].copy()]
    for t in range(40):
        n = int(rng.integers(1, 10241))
        k = rng.integers(0, int(rng.integers(1, 80)), size=n).astype(float)
        if t % 3 == 0:
            k = rng.random(n)
        if t % 5 == 0:
            k = np.sort(k)
        cases.append(k)
    for k in cases:
        assert np.array_equal(ctx.sort_order(k), O.std_sort_order(k)), k.size


def test_f4_bnb_fixture(ctx, golden_dir, f1):
    """FAST (branch-and-bound, correlate_scan_matcher.h:271-502) on the F1
    inputs: device-scored tree + host replay of the search, bit-exact."""
    f4 = np.load(os.path.join(golden_dir, "f4_bnb.npz"))
    ctx.set_grid(_map(f1["grid"], f1["resolution"], f1["offset"]), force=True)
    pose = np.array(f1["init_pose"], dtype=np.float64)
    cov = np.eye(3).reshape(9).copy()
    r = ctx.scan_match(f1["points"], _param(f4["param"]), pose, cov)
    assert r == f4["response"]
    assert np.array_equal(pose, f4["pose"]) and np.array_equal(cov, f4["cov"])


@pytest.mark.parametrize("grid_kind,depth,U", [("blur", 4, 100), ("blur", 2, 1081), ("values", 3, 50),
                                               ("hostile", 4, 100), ("flat", 4, 100), ("blur", 0, 100)])
def test_bnb_matches_oracle(ctx, f1, grid_kind, depth, U):
    """FAST on several grids / depths, incl. a flat grid (every node ties:
    the search order and std::sort decide) and depth 0 (no search)."""
    from roborts_csm import worlds
    from roborts_csm.params import FAST_PARAM
    rng = np.random.default_rng(depth * 31 + U)
    if grid_kind == "blur":
        g = f1["grid"]
    elif grid_kind == "hostile":
        g = worlds.hostile_grid(400, 400)
    elif grid_kind == "flat":
        g = np.full((400, 400), 0.3, dtype=np.float32)
    else:
        g = rng.choice(np.array([0.3, 0.41, 0.88, 1.0], dtype=np.float32), size=(400, 400))
    p = FAST_PARAM.with_(max_depth=depth, use_point_size=U)
    ctx.set_grid(_map(g, f1["resolution"], f1["offset"]), force=True)
    m = O.Map(g, float(f1["resolution"]), tuple(f1["offset"]))
    for k in range(3):
        init = np.array(f1["init_pose"], dtype=np.float64) + np.array([0.03 * k, -0.02 * k, 0.01 * k])
        pose, cov = init.copy(), np.eye(3).reshape(9).copy()
        r = ctx.scan_match(f1["points"], p, pose, cov)
        r2, pose2, cov2, _, _ = O.scan_match(m, f1["points"], p, init, np.eye(3))
        assert r == r2, (grid_kind, depth, k)
        assert np.array_equal(pose, pose2) and np.array_equal(cov, cov2), (grid_kind, depth, k)


def test_bnb_batch_matches_single(ctx, world2000):
    """csm_scan_match_batch with FAST params: each scan as if alone."""
    from roborts_csm.params import FAST_PARAM
    w, b = world2000
    ctx.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
    n = 6
    poses = np.ascontiguousarray(b.init_poses[:n].copy())
    covs = np.tile(np.eye(3).reshape(1, 9), (n, 1))
    r, _ = ctx.scan_match_batch(b.points_cells[:b.offsets[n]], b.offsets[:n + 1], FAST_PARAM, poses, covs)
    m = O.Map(w.grid, w.resolution, w.offset)
    for k in range(n):
        pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
        r2, pose2, cov2, _, _ = O.scan_match(m, pts, FAST_PARAM, b.init_poses[k], np.eye(3))
        assert r[k] == r2 and np.array_equal(poses[k], pose2) and np.array_equal(covs[k], cov2)


def test_grid_stack_best_windows(f1):
    """Loop-closure shard: submaps resident as a stack, one launch scores a
    scan in a large window on every submap (csm_best_windows), each argmax
    equal to the oracle's; the rank-local reduction of ShardedLoopClosure
    then picks the lowest global index among equal scores."""
    import roborts_csm
    from roborts_csm.loop_closure import ShardedLoopClosure, world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    rng = np.random.default_rng(41)
    base = np.stack([f1["grid"], np.roll(f1["grid"], 37, axis=0), np.roll(f1["grid"], -53, axis=1),
                     rng.choice(np.array([0.3, 0.5, 1.0], dtype=np.float32), size=f1["grid"].shape)])
    grids = np.concatenate([base, base[2:3]])  # submap 4 == submap 2: cross-submap ties
    res = float(f1["resolution"])
    offsets = np.tile(np.asarray(f1["offset"], dtype=np.float64), (grids.shape[0], 1))
    p = CorrelationScanMatchParam(2.0, 0.05, math.pi / 2, 0.0349, 0.5, 100, 0, False, 0)
    c = roborts_csm.Context(0)
    try:
        c.set_grid_stack(grids, res, version=3)
        centers = np.stack([world_to_map(f1["init_pose"], res, o) for o in offsets])
        sc, flat, x, y, a = c.best_windows(f1["points"], p, np.arange(grids.shape[0]), centers)
        for g in range(grids.shape[0]):
            m = O.Map(grids[g], res, tuple(offsets[g]))
            s2, fl2 = O.best_window(m, f1["points"], p, centers[g])
            assert sc[g] == s2 and flat[g] == fl2, g
        assert sc[4] == sc[2] and flat[4] == flat[2]
        lc = ShardedLoopClosure(c, grids.shape[0], res, offsets)
        r = lc.match(f1["points"], p, f1["init_pose"])
        na, ns = roborts_csm.window_dims(p)
        gidx = np.arange(grids.shape[0]) * (na * ns * ns) + flat
        k = int(np.argmin(np.where(sc == sc.max(), gidx, np.iinfo(np.int64).max)))
        assert r.score == sc.max() and r.global_index == gidx[k] and r.submap == k
    finally:
        c.close()


@pytest.fixture(scope="module")
def willow():
    from roborts_csm import worlds
    w = worlds.willow_world()
    b = worlds.make_scan_batch(w, 24, seed=5)
    return w, b


@pytest.mark.parametrize("which", ["sim", "headline"])
def test_willow_three_level_bit_exact(ctx, willow, which):
    """Config 4 map (the reference's willow-full-0.05, padded): batched
    3-level matching, bit-exact against the oracle."""
    from roborts_csm.params import SIM_YAML_LEVELS, headline_levels
    w, b = willow
    levels = SIM_YAML_LEVELS if which == "sim" else headline_levels()
    ctx.set_grid(_map(w.grid, w.resolution, w.offset, version=11))
    poses = np.ascontiguousarray(b.init_poses.copy())
    covs = np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1))
    s = ctx.scan_matchers_batch(b.points_cells, b.offsets, levels, poses, covs)
    m = O.Map(w.grid, w.resolution, w.offset)
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, levels, b.init_poses,
                                       np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1)))
    assert np.array_equal(s, s2) and np.array_equal(poses, p2) and np.array_equal(covs, c2)


def test_willow_best_window(ctx, willow):
    """Config 4 shape at test size: a 3 m / +-45 deg window, B = all beams."""
    from roborts_csm.params import CorrelationScanMatchParam
    w, b = willow
    ctx.set_grid(_map(w.grid, w.resolution, w.offset, version=11))
    m = O.Map(w.grid, w.resolution, w.offset)
    p = CorrelationScanMatchParam(3.0, 0.05, math.pi / 4, 0.0349, 0.5, 1081, 0, False, 0)
    for k in range(2):
        pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
        c = O.world_to_map(m, b.init_poses[k])
        got = ctx.best_window(pts, p, c)
        s, flat = O.best_window(m, pts, p, c)
        assert got.score == s and got.flat_index == flat


@pytest.mark.parametrize("finish,parts,first", [("device", 2, "0"), ("host", 2, "0"), ("device", 3, "0"),
                                                 ("device", 4, "0"), ("device", 2, "5"), ("device", 3, "1"),
                                                 ("host", 2, "5")])
def test_pipelined_three_level_driver(world2000, finish, parts, first):
    """The batch split into 2-4 parts in flight (CSM_PIPELINE threshold
    lowered so 96 scans split), the first part's coarse level launched in two
    spans (CSM_FIRST_WINDOWS, level_begin_split) or in one: results equal the
    oracle's bit for bit."""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    env = {"CSM_PIPELINE": "16", "CSM_PIPELINE_PARTS": str(parts), "CSM_FINISH": finish, "CSM_FIRST_WINDOWS": first}
    os.environ.update(env)
    try:
        c = roborts_csm.Context(0)
    finally:
        for k in env:
            del os.environ[k]
    try:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
        poses = np.ascontiguousarray(b.init_poses.copy())
        covs = np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1))
        c.set_profiling(True)
        s = c.scan_matchers_batch(b.points_cells, b.offsets, headline_levels(), poses, covs)
        st = {k["name"]: k["launches"] for k in c.kernel_stats()}
        c.set_profiling(False)
        m = O.Map(w.grid, w.resolution, w.offset)
        s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, headline_levels(), b.init_poses,
                                           np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1)))
        assert np.array_equal(s, s2) and np.array_equal(poses, p2) and np.array_equal(covs, c2)
        assert st["host:wait"] == 3 * parts  # 3 levels x parts
    finally:
        c.close()


def test_host_signal_split_levels_with_ties(world2000):
    """Host-signal finish where the exact pass has work on every level: a map
    quantised to three values makes equal scores common, so windows of the
    coarse level too go to the exact pass. The first part's coarse level runs
    in two scoring spans and a finish-only call (level_begin_split); the list
    of flagged windows carries the tag of the slot's latest scoring call, and
    the scoring does not wait for the slot's previous exact pass (a stale one
    finds another tag). Twenty batches back to back: each equals the oracle's
    answer bit for bit. (r04: the host completed settled windows from
    FinishOut pieces that had not landed yet -- 2-16 of 60 batches -- until
    every window carried a checked seal; tools/stress_ties.py.)"""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    grid = np.round(np.asarray(w.grid, dtype=np.float32) * 2.0).astype(np.float32) / np.float32(2.0)
    # growing first-level spans from 5 windows, the last part's hand-off to
    # the super-fine level in two spans (from parts of 8 windows)
    env = {"CSM_PIPELINE": "16", "CSM_PIPELINE_PARTS": "2", "CSM_FIRST_WINDOWS": "5", "CSM_SPLIT_HANDOFF_MIN": "8"}
    os.environ.update(env)
    try:
        c = roborts_csm.Context(0)
    finally:
        for k in env:
            del os.environ[k]
    m = O.Map(grid, w.resolution, w.offset)
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, headline_levels(), b.init_poses,
                                       np.tile(np.eye(3).reshape(1, 9), (b.init_poses.shape[0], 1)))
    try:
        c.set_grid(_map(grid, w.resolution, w.offset, version=1))
        c.set_profiling(True)
        for it in range(20):
            poses = np.ascontiguousarray(b.init_poses.copy())
            covs = np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1))
            s = c.scan_matchers_batch(b.points_cells, b.offsets, headline_levels(), poses, covs)
            assert np.array_equal(s, s2) and np.array_equal(poses, p2) and np.array_equal(covs, c2), it
        st = {k["name"]: k for k in c.kernel_stats()}
        c.set_profiling(False)
        coarse = [k for n, k in st.items() if n.startswith("finish:exact_windows<") and "5070" in n]
        assert coarse and coarse[0]["scorings"] > 0  # the coarse level's exact pass had windows
    finally:
        c.close()


def test_host_signal_finish_repeated(world2000):
    """The throughput path's host-signal finish (FinishOut written through to
    coherent host memory, a flag instead of a D2H copy and an event) over 25
    back-to-back 3-level batches in 2 parts: every batch equals the oracle's
    answer bit for bit, and the copy-back path (CSM_HOST_SIGNAL=0) agrees."""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    m = O.Map(w.grid, w.resolution, w.offset)
    eye = np.tile(np.eye(3).reshape(1, 9), (b.init_poses.shape[0], 1))
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, headline_levels(), b.init_poses, eye.copy())
    for sig in ("1", "0"):
        env = {"CSM_PIPELINE": "16", "CSM_HOST_SIGNAL": sig, "CSM_FIRST_WINDOWS": "8"}
        os.environ.update(env)
        try:
            c = roborts_csm.Context(0)
        finally:
            for k in env:
                del os.environ[k]
        try:
            c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
            c.load_scans(b.points_cells, b.offsets)
            for it in range(25 if sig == "1" else 3):
                poses = np.ascontiguousarray(b.init_poses.copy())
                covs = eye.copy()
                s = c.scan_matchers_loaded(headline_levels(), poses, covs)
                assert np.array_equal(s, s2) and np.array_equal(poses, p2) and np.array_equal(covs, c2), (sig, it)
        finally:
            c.close()


@pytest.mark.parametrize("order,use_fine", [((0, 1, 2), True), ((0, 1, 2), False), ((1, 0, 2), True),
                                            ((0, 2, 1), True), ((2, 2, 0), True)])
def test_dead_covariance_lists_skipped_exactly(world2000, order, use_fine):
    """The 3-level driver fills only the covariance lists a later level does
    not overwrite (live_lists: the fine level's ComputePositionalCovariance
    resets the matrix, :891). Device finish + pipelined driver, the default
    and CSM_SKIP_DEAD_LISTS=0, and odd level orders: all equal the oracle."""
    import roborts_csm
    from roborts_csm.params import SIM_YAML_LEVELS, headline_levels
    w, b = world2000
    base = headline_levels()
    # level k takes the window of headline level k and the type of order[k]
    levels = tuple(base[k].with_(correlation_scan_match_type=SIM_YAML_LEVELS[order[k]].correlation_scan_match_type)
                   for k in range(3))
    m = O.Map(w.grid, w.resolution, w.offset)
    eye = np.tile(np.eye(3).reshape(1, 9), (b.init_poses.shape[0], 1))
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, levels, b.init_poses, eye.copy(),
                                       use_fine=use_fine)
    for skip in ("1", "0"):
        os.environ["CSM_PIPELINE"] = "16"
        os.environ["CSM_FINISH"] = "device"
        os.environ["CSM_SKIP_DEAD_LISTS"] = skip
        try:
            c = roborts_csm.Context(0)
        finally:
            for k in ("CSM_PIPELINE", "CSM_FINISH", "CSM_SKIP_DEAD_LISTS"):
                del os.environ[k]
        try:
            c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
            poses = np.ascontiguousarray(b.init_poses.copy())
            covs = eye.copy()
            s = c.scan_matchers_batch(b.points_cells, b.offsets, levels, poses, covs, use_fine=use_fine)
            assert np.array_equal(s, s2) and np.array_equal(poses, p2) and np.array_equal(covs, c2), skip
        finally:
            c.close()


@pytest.mark.parametrize("margin_log2,thin", [(None, 1), ("5", 1), (None, 10), ("5", 10)])
def test_phase_kernel_edge_beams(world2000, margin_log2, thin):
    """v7 phase kernel (sub-cell window step) on its margin cases: beams whose
    phase sits on or near a bucket edge (origin points with window phases at
    the breakpoints 0, 0.2, 0.4, ...), beams off the grid's low edge (negative
    t) and past its high edges, windows at inexact step sums; with the default
    2^-20 margin and with a 1/32 margin that sends ~half the beams down the exact
    path. All scores and the argmax against the oracle and the v4 row kernel;
    the phase kernel over the strip copies of gridi (default) and over gridi
    itself (CSM_PHASE_STRIPS=0). thin = 10: every 10th beam plus the edge
    beams, 119 in all: the short-scan form (kPhaseShortBeams, two chunks a
    segment)."""
    import roborts_csm
    from roborts_csm.params import SIM_YAML_LEVELS
    w, b = world2000
    m = O.Map(w.grid, w.resolution, w.offset)
    pts = b.points_cells[b.offsets[0]:b.offsets[1]][::thin]
    extra = np.array([[0.0, 0.0], [0.0, 0.0], [1.0, -2.0], [-1500.0, 3.0], [2.0, -1500.0],
                      [900.0, 900.0], [-3000.0, -3000.0], [0.25, 0.0], [0.2, 0.6], [-0.4, 0.8]])
    pts = np.ascontiguousarray(np.concatenate([pts, extra]))
    lv = SIM_YAML_LEVELS[1].with_(use_point_size=pts.shape[0])
    half = (lv.search_space_size / w.resolution) * 0.5
    centers = [[100.5 + half, 200.5 + half, 0.0], [100.7 + half, 200.9 + half, 1.3],
               [100.3 + half, 200.1 + half, -0.4],
               [1020.0 + 3 * 2.0 ** -43, 1019.0 + 2.0 ** -43, 0.7],
               [1.2, 0.1, -2.5], [1998.0, 1990.0, 1.0], [511.0 + 2.0 ** -44, 250.3, 3.0]]
    env = {"CSM_PHASE_MARGIN_LOG2": margin_log2} if margin_log2 else {}
    ctxs = [_variant_ctx(k, **env) for k in (None, "v4", "split")] + [_variant_ctx(None, CSM_PHASE_STRIPS="0",
                                                                                **env)]
    for c in ctxs:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
    ctxs[0].set_profiling(True)
    ctxs[3].set_profiling(True)
    for cen in centers:
        cen = np.array(cen)
        want = O.score_window(m, pts, lv, cen, 11 * 11 * 11)
        for c in ctxs:
            assert np.array_equal(c.score_window(pts, lv, cen), want), cen
            got = c.best_window(pts, lv, cen)
            s, flat = O.best_window(m, pts, lv, cen)
            assert got.score == s and got.flat_index == flat
    for i, strips in ((0, True), (3, False)):
        names = {k["name"] for k in ctxs[i].kernel_stats()}
        assert "score_phase_kernel<11,all>" in names and "score_phase_kernel<11,best>" in names, names
        assert ("grid:istrips" in names) == strips, names
    for c in ctxs:
        c.close()


def test_phase_kernel_low_edge_straddle(world2000):
    """Fine-level (v7 phase) windows whose boxes straddle the grid's low edges:
    the reference truncates toward zero (a cell coordinate in (-1, 0) reads
    row / column 0, one at or below -1 the outside value); the phase strips
    hold that in their low-side padding (column -1 repeats column 0, row -1
    row 0). Row 0 and column 0 carry values found nowhere else. Scores and
    argmax against the oracle, over the strips and over gridi itself."""
    w, _ = world2000
    rng = np.random.default_rng(31)
    vals = np.array([0.3, 0.375, 0.5, 0.625, 0.75], dtype=np.float32)
    g = rng.choice(vals, size=(300, 300)).astype(np.float32)
    g[0, :] = np.float32(0.875)
    g[:, 0] = np.float32(1.0)
    g[0, 0] = np.float32(0.4375)
    res = w.resolution
    m = O.Map(g, res, (0.0, 0.0))
    from roborts_csm.params import SIM_YAML_LEVELS
    pts = np.ascontiguousarray(rng.uniform(-7.0, 7.0, size=(600, 2)))
    pts[:30] = np.round(pts[:30] * 5.0) / 5.0  # fifth cells: phases on bucket edges
    lv = SIM_YAML_LEVELS[1].with_(use_point_size=pts.shape[0])
    centers = [np.array([rng.uniform(-4.0, 8.0), rng.uniform(-4.0, 8.0), rng.uniform(-np.pi, np.pi)])
               for _ in range(8)]
    centers += [np.array([2.0, 150.0, 0.3]), np.array([150.0, 1.5, -1.0])]
    ctxs = [_variant_ctx(None), _variant_ctx(None, CSM_PHASE_STRIPS="0")]
    for c in ctxs:
        c.set_grid(_map(g, res, (0.0, 0.0), version=1))
        c.set_profiling(True)
    try:
        for cen in centers:
            want = O.score_window(m, pts, lv, cen, 11 * 11 * 11)
            s, flat = O.best_window(m, pts, lv, cen)
            for c in ctxs:
                assert np.array_equal(c.score_window(pts, lv, cen), want), cen
                got = c.best_window(pts, lv, cen)
                assert got.score == s and got.flat_index == flat, cen
        names = {k["name"] for k in ctxs[0].kernel_stats()}
        assert "score_phase_kernel<11,all>" in names and "grid:istrips" in names, names
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("size,res", [(0.02, 0.01), (0.01, 0.01), (0.03, 0.01), (0.015, 0.005)])
def test_tiny_kernel_edge_beams(world2000, size, res):
    """v8 tiny-window kernel (spans under one cell: the super-fine level, 3 x 3
    steps of 0.2 cells, and 2 x 2 / 4 x 4 / 0.1-cell variants) on its edge
    cases: origin points on rounding boundaries, beams off the grid's low edge
    (negative indices: the cell-by-cell path) and far past the high edges,
    windows at inexact step sums, every beam summed (several 16-chunk folds).
    Scores and argmax against the oracle and the v4 row kernel."""
    import roborts_csm
    from roborts_csm.params import SIM_YAML_LEVELS
    w, b = world2000
    m = O.Map(w.grid, w.resolution, w.offset)
    pts = np.concatenate([b.points_cells[b.offsets[k]:b.offsets[k + 1]] for k in range(2)])
    extra = np.array([[0.0, 0.0], [0.0, 0.0], [1.0, -2.0], [-1500.0, 3.0], [2.0, -1500.0],
                      [900.0, 900.0], [-3000.0, -3000.0], [0.25, 0.0], [0.2, 0.6], [-0.4, 0.8],
                      [0.5, 0.5], [-0.5, -0.5]])
    pts = np.ascontiguousarray(np.concatenate([pts, extra]))
    lv = SIM_YAML_LEVELS[2].with_(search_space_size=size, search_space_resolution=res,
                                  use_point_size=pts.shape[0])
    na, ns = roborts_csm.window_dims(lv)
    assert 2 <= ns <= 4
    half = (lv.search_space_size / w.resolution) * 0.5
    centers = [[100.5 + half, 200.5 + half, 0.0], [100.7 + half, 200.9 + half, 1.3],
               [100.3 + half, 200.1 + half, -0.4], [1020.0 + 3 * 2.0 ** -43, 1019.0 + 2.0 ** -43, 0.7],
               [0.2, 0.1, -2.5], [1999.6, 1999.7, 1.0], [511.0 + 2.0 ** -44, 250.3, 3.0]]
    ctxs = [_variant_ctx(k) for k in (None, "v4", "split")]
    for c in ctxs:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
    ctxs[0].set_profiling(True)
    for cen in centers:
        cen = np.array(cen)
        want = O.score_window(m, pts, lv, cen, na * ns * ns)
        for c in ctxs:
            assert np.array_equal(c.score_window(pts, lv, cen), want), cen
            got = c.best_window(pts, lv, cen)
            s, flat = O.best_window(m, pts, lv, cen)
            assert got.score == s and got.flat_index == flat
    names = {k["name"] for k in ctxs[0].kernel_stats()}
    assert f"score_tiny_kernel<{ns},all>" in names and f"score_tiny_kernel<{ns},best>" in names, names
    for c in ctxs:
        c.close()


def test_phase_kernel_batch_segments(world2000):
    """Scans longer than one classification segment (1152 beams, every beam
    summed) and short ones in one phase launch, against the oracle."""
    from roborts_csm.params import SIM_YAML_LEVELS
    import roborts_csm
    w, b = world2000
    m = O.Map(w.grid, w.resolution, w.offset)
    rng = np.random.default_rng(5)
    scans = [np.ascontiguousarray(np.concatenate([b.points_cells[b.offsets[k]:b.offsets[k + 1]]] * r))
             for k, r in ((0, 3), (1, 1), (2, 2))]
    scans.append(rng.uniform(-60, 60, size=(7, 2)))
    c = _variant_ctx(None)
    try:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
        for pts in scans:
            lv = SIM_YAML_LEVELS[1].with_(use_point_size=pts.shape[0])
            cen = O.world_to_map(m, b.init_poses[0])
            assert np.array_equal(c.score_window(pts, lv, cen), O.score_window(m, pts, lv, cen, 1331))
    finally:
        c.close()


def test_load_scans_async_queue(world2000):
    """csm_load_scans_async: batches queued from pinned host memory (two at a
    time), each taken by the next csm_scan_matchers_loaded, equal the oracle's
    answer bit for bit; a third queued batch is refused."""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    m = O.Map(w.grid, w.resolution, w.offset)
    n = 48
    halves = [(0, n), (n, 2 * n)]
    pins, offs, want = [], [], []
    for lo, hi in halves:
        pts = b.points_cells[b.offsets[lo]:b.offsets[hi]]
        p = roborts_csm.PinnedArray(pts.shape)
        np.copyto(p.array, pts)
        pins.append(p)
        off = np.ascontiguousarray(b.offsets[lo:hi + 1] - b.offsets[lo])
        offs.append(off)
        eye = np.tile(np.eye(3).reshape(1, 9), (hi - lo, 1))
        want.append(O.scan_matchers_batch(m, pts, off, headline_levels(), b.init_poses[lo:hi], eye.copy()))
    env = {"CSM_PIPELINE": "16"}
    os.environ.update(env)
    try:
        c = roborts_csm.Context(0)
    finally:
        for k in env:
            del os.environ[k]
    try:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
        for rnd in range(2):
            c.load_scans_async(pins[0].array, offs[0])
            c.load_scans_async(pins[1].array, offs[1])
            if rnd == 0:
                with pytest.raises(roborts_csm.CsmError):
                    c.load_scans_async(pins[0].array, offs[0])
            for (lo, hi), (s2, p2, c2) in zip(halves, want):
                poses = np.ascontiguousarray(b.init_poses[lo:hi].copy())
                covs = np.tile(np.eye(3).reshape(1, 9), (hi - lo, 1))
                s = c.scan_matchers_loaded(headline_levels(), poses, covs)
                assert np.array_equal(s, s2) and np.array_equal(poses, p2) and np.array_equal(covs, c2), (rnd, lo)
    finally:
        c.close()
        for p in pins:
            p.close()


@pytest.mark.parametrize("quantised,defer", [(False, "1"), (True, "1"), (True, "0")])
def test_submitted_batches_equal_loaded(world2000, quantised, defer):
    """csm_scan_matchers_submit: batches in flight back to back (a batch's
    last level completed while the next one's first launch scores, in the
    other half of the buffer slots) give csm_scan_matchers_loaded's answers
    bit for bit; a synchronous call in between completes the pending batch
    first; on the 3-value map every level's exact pass has windows."""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    grid = w.grid
    if quantised:
        grid = np.round(np.asarray(w.grid, dtype=np.float32) * 2.0).astype(np.float32) / np.float32(2.0)
    env = {"CSM_PIPELINE": "16", "CSM_PIPELINE_PARTS": "2", "CSM_FIRST_WINDOWS": "5", "CSM_SPLIT_HANDOFF_MIN": "8",
           "CSM_DEFER_HANDOFF": defer}
    os.environ.update(env)
    try:
        c = roborts_csm.Context(0)
    finally:
        for k in env:
            del os.environ[k]
    try:
        c.set_grid(_map(grid, w.resolution, w.offset, version=1))
        c.load_scans(b.points_cells, b.offsets)
        n = b.init_poses.shape[0]
        rng = np.random.default_rng(3)
        inits = [np.ascontiguousarray(b.init_poses + rng.uniform(-1, 1, size=(n, 3)) * [0.05, 0.05, 0.02])
                 for _ in range(5)]
        eye = np.tile(np.eye(3).reshape(1, 9), (n, 1))
        want = []
        for p0 in inits:
            p, cv = p0.copy(), eye.copy()
            s = c.scan_matchers_loaded(headline_levels(), p, cv)
            want.append((s, p, cv))
        got = [(np.zeros(n), p0.copy(), eye.copy()) for p0 in inits]
        for k in (0, 1):
            c.scan_matchers_submit(headline_levels(), got[k][1], got[k][2], got[k][0])
        p, cv = inits[2].copy(), eye.copy()  # completes batch 1 first
        s = c.scan_matchers_loaded(headline_levels(), p, cv)
        got[2] = (s, p, cv)
        for k in (3, 4):
            c.scan_matchers_submit(headline_levels(), got[k][1], got[k][2], got[k][0])
        c.scan_matchers_wait()
        for k in range(5):
            for a, e in zip(got[k], want[k]):
                assert np.array_equal(a, e), k
    finally:
        c.close()


@pytest.mark.parametrize("first_windows", ["5", None])
def test_submitted_batches_from_staged_scans(world2000, first_windows):
    """csm_load_scans_async + csm_scan_matchers_submit, a different batch of
    scans per submit: the queued batch is taken while the previous one is
    still pending (its points parked in a staging slot until it completes),
    and every batch's answers equal its own synchronous load + match."""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    env = {"CSM_PIPELINE": "16", "CSM_PIPELINE_PARTS": "2", "CSM_SPLIT_HANDOFF_MIN": "8"}
    if first_windows is not None:  # None: the submitted batches' own defaults (one first launch, 50/50)
        env["CSM_FIRST_WINDOWS"] = first_windows
    os.environ.update(env)
    try:
        c = roborts_csm.Context(0)
    finally:
        for k in env:
            del os.environ[k]
    n = b.init_poses.shape[0]
    eye = np.tile(np.eye(3).reshape(1, 9), (n, 1))
    batches = [np.ascontiguousarray(b.points_cells * f) for f in (1.0, 0.98, 1.02, 0.99, 1.01)]
    pins = []
    try:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
        want = []
        for q in batches:
            c.load_scans(q, b.offsets)
            p, cv = b.init_poses.copy(), eye.copy()
            want.append((c.scan_matchers_loaded(headline_levels(), p, cv), p, cv))
        for q in batches:
            pins.append(roborts_csm.PinnedArray(q.shape))
            np.copyto(pins[-1].array, q)
        got = [(np.zeros(n), b.init_poses.copy(), eye.copy()) for _ in batches]
        c.load_scans_async(pins[0].array, b.offsets)
        for k in range(len(batches)):
            if k + 1 < len(batches):
                c.load_scans_async(pins[k + 1].array, b.offsets)
            c.scan_matchers_submit(headline_levels(), got[k][1], got[k][2], got[k][0])
        c.scan_matchers_wait()
        for k in range(len(batches)):
            for a, e in zip(got[k], want[k]):
                assert np.array_equal(a, e), k
    finally:
        c.close()
        for p in pins:
            p.close()


def test_sync_entry_points_drop_queued_batches(world2000):
    """A batch queued with csm_load_scans_async is dropped, not matched, by
    the calls that load their own scans (csm_scan_matchers,
    csm_scan_matchers_batch, csm_load_scans): each returns its own scans'
    answers (the r04 driver handed them the queued batch's, written into
    arrays sized for their own scans). A batch queued afterwards is still
    taken by the next csm_scan_matchers_loaded."""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    m = O.Map(w.grid, w.resolution, w.offset)
    lv = headline_levels()
    other = np.ascontiguousarray(b.points_cells * 0.98)
    pin = roborts_csm.PinnedArray(other.shape)
    np.copyto(pin.array, other)
    c = roborts_csm.Context(0)
    try:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
        # one scan
        c.load_scans_async(pin.array, b.offsets)
        one = b.points_cells[b.offsets[0]:b.offsets[1]]
        pose, cov = b.init_poses[0].copy(), np.eye(3).reshape(9).copy()
        s = c.scan_matchers(one, lv, pose, cov)
        s2, p2, c2 = O.scan_matchers(m, one, lv, b.init_poses[0], np.eye(3).reshape(9))
        assert s == s2 and np.array_equal(pose, p2) and np.array_equal(cov, c2)
        # a batch of 8
        c.load_scans_async(pin.array, b.offsets)
        c.load_scans_async(pin.array, b.offsets)
        n = 8
        sub = b.points_cells[:b.offsets[n]]
        off = np.ascontiguousarray(b.offsets[:n + 1])
        eye = np.tile(np.eye(3).reshape(1, 9), (n, 1))
        poses = np.ascontiguousarray(b.init_poses[:n].copy())
        covs = eye.copy()
        s = c.scan_matchers_batch(sub, off, lv, poses, covs)
        s2, p2, c2 = O.scan_matchers_batch(m, sub, off, lv, b.init_poses[:n], eye.copy())
        assert np.array_equal(s, s2) and np.array_equal(poses, p2) and np.array_equal(covs, c2)
        # csm_load_scans drops the queue too; the loaded call runs the loaded scans
        c.load_scans_async(pin.array, b.offsets)
        c.load_scans(sub, off)
        poses, covs = np.ascontiguousarray(b.init_poses[:n].copy()), eye.copy()
        s = c.scan_matchers_loaded(lv, poses, covs)
        assert np.array_equal(s, s2) and np.array_equal(poses, p2) and np.array_equal(covs, c2)
        # queued after the synchronous calls: taken
        nb = b.init_poses.shape[0]
        c.load_scans_async(pin.array, b.offsets)
        poses, covs = np.ascontiguousarray(b.init_poses.copy()), np.tile(np.eye(3).reshape(1, 9), (nb, 1))
        s = c.scan_matchers_loaded(lv, poses, covs)
        s3, p3, c3 = O.scan_matchers_batch(m, other, b.offsets, lv, b.init_poses,
                                           np.tile(np.eye(3).reshape(1, 9), (nb, 1)))
        assert np.array_equal(s, s3) and np.array_equal(poses, p3) and np.array_equal(covs, c3)
    finally:
        c.close()
        pin.close()


def test_submitted_batches_of_varied_sizes(world2000):
    """Queued batches of different scan counts submitted back to back, one
    below CSM_PIPELINE (the synchronous fallback between pipelined submits,
    which completes the pending batch on its parked points): every batch
    equals its own synchronous load + match."""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    env = {"CSM_PIPELINE": "16", "CSM_PIPELINE_PARTS": "2"}
    os.environ.update(env)
    try:
        c = roborts_csm.Context(0)
    finally:
        for k in env:
            del os.environ[k]
    lv = headline_levels()
    sizes, scales = (96, 40, 10, 96, 64, 17), (1.0, 0.98, 1.02, 0.99, 1.01, 0.97)
    batches = []
    for n, f in zip(sizes, scales):
        off = np.ascontiguousarray(b.offsets[:n + 1])
        batches.append((np.ascontiguousarray(b.points_cells[:b.offsets[n]] * f), off, n))
    pins = []
    try:
        c.set_grid(_map(w.grid, w.resolution, w.offset, version=1))
        want = []
        for q, off, n in batches:
            c.load_scans(q, off)
            p, cv = b.init_poses[:n].copy(), np.tile(np.eye(3).reshape(1, 9), (n, 1))
            want.append((c.scan_matchers_loaded(lv, p, cv), p, cv))
        for q, _, _ in batches:
            pins.append(roborts_csm.PinnedArray(q.shape))
            np.copyto(pins[-1].array, q)
        got = [(np.zeros(n), b.init_poses[:n].copy(), np.tile(np.eye(3).reshape(1, 9), (n, 1)))
               for _, _, n in batches]
        c.load_scans_async(pins[0].array, batches[0][1])
        for k in range(len(batches)):
            if k + 1 < len(batches):
                c.load_scans_async(pins[k + 1].array, batches[k + 1][1])
            c.scan_matchers_submit(lv, got[k][1], got[k][2], got[k][0])
        c.scan_matchers_wait()
        for k in range(len(batches)):
            for a, e in zip(got[k], want[k]):
                assert np.array_equal(a, e), (k, sizes[k])
    finally:
        c.close()
        for p in pins:
            p.close()


@pytest.fixture(scope="module")
def world2000_bench():
    """The bench's own config-2 inputs: the seeded 2000 x 2000 world and
    rank 0's 4096-scan batch (bench.py main)."""
    from roborts_csm import worlds
    w = worlds.make_world(2000, 2000, 0.05, seed=20261015)
    b = worlds.make_scan_batch(w, 4096, seed=1000)
    return w, b


@pytest.mark.parametrize("quantised,levels", [(False, "headline"), (True, "headline"), (False, "sim"), (True, "sim")])
def test_timed_configuration_against_oracle(world2000_bench, quantised, levels):
    """The configuration bench.py times, with no CSM_* overrides: 4096 scans
    (two parts of 2048 windows), batches queued from pinned host memory
    (csm_load_scans_async) and submitted back to back with the library's
    submitted-batch defaults (a 512-window first coarse span at B = 1081,
    50/50 part split, deferred last hand-off). Three different batches, each
    against the
    oracle bit for bit (scores, poses, covariances); on the 3-value map
    every level's exact pass has windows. Both beam rules: every beam (B =
    1081, the headline) and the sim YAML's U = 100 (B = 109), whose levels
    finish their windows inside the scoring launches (csm_tail.hpp)."""
    import roborts_csm
    from roborts_csm.params import SIM_YAML_LEVELS, headline_levels
    w, b = world2000_bench
    grid = w.grid
    if quantised:
        grid = np.round(np.asarray(w.grid, dtype=np.float32) * 2.0).astype(np.float32) / np.float32(2.0)
    assert not any(k.startswith("CSM_") for k in os.environ), "the defaults are under test"
    lv = headline_levels() if levels == "headline" else SIM_YAML_LEVELS
    n = b.init_poses.shape[0]
    eye = np.tile(np.eye(3).reshape(1, 9), (n, 1))
    rng = np.random.default_rng(11)
    scans = [np.ascontiguousarray(b.points_cells * f) for f in (1.0, 0.995, 1.005)]
    inits = [np.ascontiguousarray(b.init_poses + rng.uniform(-1, 1, size=(n, 3)) * [0.03, 0.03, 0.01])
             for _ in scans]
    m = O.Map(grid, w.resolution, w.offset)
    O.set_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    try:
        want = [O.scan_matchers_batch(m, q, b.offsets, lv, p0, eye.copy()) for q, p0 in zip(scans, inits)]
    finally:
        O.set_threads(1)
    c = roborts_csm.Context(0)
    pins = []
    try:
        c.set_grid(_map(grid, w.resolution, w.offset, version=1))
        for q in scans:
            pins.append(roborts_csm.PinnedArray(q.shape))
            np.copyto(pins[-1].array, q)
        got = [(np.zeros(n), p0.copy(), eye.copy()) for p0 in inits]
        c.set_profiling(True)
        c.load_scans_async(pins[0].array, b.offsets)
        for k in range(len(scans)):
            if k + 1 < len(scans):
                c.load_scans_async(pins[k + 1].array, b.offsets)
            c.scan_matchers_submit(lv, got[k][1], got[k][2], got[k][0])
        c.scan_matchers_wait()
        st = {k["name"]: k for k in c.kernel_stats()}
        c.set_profiling(False)
        for k in range(len(scans)):
            s2, p2, c2 = want[k]
            assert np.array_equal(got[k][0], s2), (k, int(np.sum(got[k][0] != s2)))
            assert np.array_equal(got[k][1], p2), (k, int(np.sum(np.any(got[k][1] != p2, axis=1))))
            assert np.array_equal(got[k][2], c2), (k, int(np.sum(np.any(got[k][2] != c2, axis=1))))
        assert st["score_box_pair_kernel<13,all>"]["launches"] >= 2 * len(scans), st.keys()
        # the fused finish at B = 109 leaves no fast-pass time; B = 1081 keeps the fast pass
        fast = sum(k["total_ms"] for nm, k in st.items() if nm.startswith("finish:fast<"))
        if levels == "sim":
            assert fast < 0.02 * len(scans) * 6, fast
        else:
            assert fast > 0.005 * len(scans) * 6, fast
        if quantised:
            ex = [k for nm, k in st.items() if nm.startswith("finish:exact_windows<")]
            assert len(ex) == 3 and all(k["scorings"] > 0 for k in ex), ex
        # the bench's timed region: events around the first level's scoring launches only
        # (csm_set_profiling mode 2), the same results
        c.set_profiling(2)
        c.load_scans(scans[0], b.offsets)
        again = (np.zeros(n), inits[0].copy(), eye.copy())
        c.scan_matchers_submit(lv, again[1], again[2], again[0])
        c.scan_matchers_wait()
        st2 = {k["name"] for k in c.kernel_stats()}
        c.set_profiling(False)
        for g, e in zip(again, want[0]):
            assert np.array_equal(g, e)
        assert "score_box_pair_kernel<13,all>" in st2, st2
        assert not any(nm.startswith(("score_phase", "score_tiny")) for nm in st2), st2
    finally:
        c.close()
        for p in pins:
            p.close()
