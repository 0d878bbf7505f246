"""GPU parity of the admissible multi-resolution search (csm_search_windows,
csrc/csm_pyramid.hip) against the exhaustive device argmax (csm_best_windows,
itself pinned to the oracle) and against the CPU oracle's best_window
(oracle/csm_oracle.cpp, the reference's GetResponse loop over every
candidate, correlate_scan_matcher.h:552-583,637-662).

The bar is identity: the same score bits, the same window, the same flat
index (ties to the lowest (window, flat) index, the order the reference's
enumeration produces), the same pose. Config 3 (321^2 x 181 windows on
800 x 800 submaps) and config 4 (the willow map, 20 m window) run at their
real window sizes, and one stack puts the winner beyond global index 2^32.
"""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import pyoracle as O  # noqa: E402


def _reduce(sc, flat, n_cand):
    gidx = np.arange(sc.size, dtype=np.int64) * n_cand + flat.astype(np.int64)
    best = sc.max()
    k = int(np.argmin(np.where(sc == best, gidx, np.iinfo(np.int64).max)))
    return k, gidx[k]


def _check_same(ctx, pts, p, gi, centers, **kw):
    """search_windows == reduced best_windows; returns (best, window, stats)."""
    import roborts_csm
    na, ns = roborts_csm.window_dims(p)
    sc, flat, x, y, a = ctx.best_windows(pts, p, gi, centers)
    k, _ = _reduce(sc, flat, na * ns * ns)
    b, w, st = ctx.search_windows(pts, p, gi, centers, **kw)
    assert w == k, (w, k, st)
    assert b.score == sc[k] and b.flat_index == flat[k], (b.score, sc[k], b.flat_index, flat[k])
    assert b.x == x[k] and b.y == y[k] and b.angle == a[k]
    return b, w, st


@pytest.fixture(scope="module")
def f1(golden_dir):
    return np.load(os.path.join(golden_dir, "f1_config1.npz"))


@pytest.fixture(scope="module")
def stack5(f1):
    rng = np.random.default_rng(41)
    base = np.stack([f1["grid"], np.roll(f1["grid"], 37, axis=0), np.roll(f1["grid"], -53, axis=1),
                     rng.choice(np.array([0.3, 0.5, 1.0], dtype=np.float32), size=f1["grid"].shape)])
    return np.concatenate([base, base[2:3]])  # submap 4 == submap 2: cross-window ties


@pytest.mark.parametrize("depth", [-1, 0, 1, 3, 6])
@pytest.mark.parametrize("penalty", [False, True])
def test_search_matches_exhaustive_and_oracle(f1, stack5, depth, penalty):
    import roborts_csm
    from roborts_csm.loop_closure import world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    res = float(f1["resolution"])
    offsets = np.tile(np.asarray(f1["offset"], dtype=np.float64), (stack5.shape[0], 1))
    p = CorrelationScanMatchParam(2.0, 0.05, math.pi / 2, 0.0349, 0.5, 100, 0, penalty, 0)
    with roborts_csm.Context(0) as c:
        c.set_grid_stack(stack5, res, version=3)
        centers = np.stack([world_to_map(f1["init_pose"], res, o) for o in offsets])
        b, w, st = _check_same(c, f1["points"], p, np.arange(stack5.shape[0]), centers, max_depth=depth)
        assert not st["exhaustive"]
        if depth >= 0:
            assert st["depth"] == depth
        # the oracle's per-window argmax, reduced the same way
        na, ns = roborts_csm.window_dims(p)
        os_, of_ = zip(*[O.best_window(O.Map(stack5[g], res, tuple(offsets[g])), f1["points"], p, centers[g])
                         for g in range(stack5.shape[0])])
        k, _ = _reduce(np.array(os_), np.array(of_), na * ns * ns)
        assert w == k and b.score == os_[k] and b.flat_index == of_[k]
        # pruning did something (depth 0 is the exhaustive walk itself)
        if depth != 0:
            assert st["nodes"][0] + st["probe_leaves"] < st["candidates"]


def test_search_slices_and_probes(f1, stack5):
    """A node capacity of 64 forces every level to be expanded in slices
    (depth-first over slices), probes at every level: same answer."""
    import roborts_csm
    from roborts_csm.loop_closure import world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    res = float(f1["resolution"])
    p = CorrelationScanMatchParam(2.0, 0.05, math.pi / 4, 0.0349, 0.5, 100, 0, True, 1)
    with roborts_csm.Context(0) as c:
        c.set_grid_stack(stack5, res, version=3)
        centers = np.stack([world_to_map(f1["init_pose"], res, f1["offset"])] * stack5.shape[0])
        _check_same(c, f1["points"], p, np.arange(stack5.shape[0]), centers, max_depth=4, node_capacity=64,
                    probe_min_nodes=1)


@pytest.mark.parametrize("depth", [3, 5])
def test_search_many_slices_without_probes(f1, stack5, depth):
    """No probe anywhere (probe_min_nodes < 0) and the smallest node capacity:
    the incumbent only rises at depth 0, so almost nothing is pruned early and
    the search runs through far more than the 64 fresh list counters. Every
    slice's parent count must survive its children's counter being cleared
    (each depth's fallback counter is its own): same answer as exhaustive."""
    import roborts_csm
    from roborts_csm.loop_closure import world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    res = float(f1["resolution"])
    p = CorrelationScanMatchParam(1.6, 0.05, 0.35, 0.0349, 0.5, 100, 0, False, 0)
    with roborts_csm.Context(0) as c:
        c.set_grid_stack(stack5, res, version=3)
        centers = np.stack([world_to_map(f1["init_pose"], res, f1["offset"])] * stack5.shape[0])
        b, w, st = _check_same(c, f1["points"], p, np.arange(stack5.shape[0]), centers, max_depth=depth,
                               node_capacity=16, probe_min_nodes=-1)
        assert st["probe_leaves"] == 0
        assert st["syncs"] > 64, st  # each read-back follows an expand: > 64 expands


@pytest.mark.parametrize("penalty", [False, True])
def test_search_plateau_ties(f1, penalty):
    """Every candidate scores the same (a constant grid): the answer is the
    lowest (window, flat); with the centre penalty the centre wins."""
    import roborts_csm
    from roborts_csm.params import CorrelationScanMatchParam
    g = np.full((3,) + f1["grid"].shape, 0.5, dtype=np.float32)
    res = float(f1["resolution"])
    p = CorrelationScanMatchParam(1.0, 0.05, 0.2, 0.0349, 0.5, 100, 0, penalty, 0)
    with roborts_csm.Context(0) as c:
        c.set_outside_value(0.5)
        c.set_grid_stack(g, res, version=1)
        centers = np.array([[200.0, 200.0, 0.1]] * 3)
        b, w, st = _check_same(c, f1["points"], p, np.arange(3), centers, max_depth=3)
        if not penalty:
            assert w == 0 and b.flat_index == 0


def test_search_negative_fixed_point_and_off_grid(f1):
    """Cells below the outside value (negative fixed-point values: the
    penalised bound's < 0 branch), windows hanging off the grid's edges."""
    import roborts_csm
    from roborts_csm.params import CorrelationScanMatchParam
    rng = np.random.default_rng(7)
    g = rng.choice(np.array([0.0, 0.25, 0.5, 1.0], dtype=np.float32), size=(2,) + f1["grid"].shape)
    res = float(f1["resolution"])
    sy, sx = g.shape[1:]
    for penalty in (False, True):
        p = CorrelationScanMatchParam(3.0, 0.05, 0.5, 0.0349, 0.5, 100, 0, penalty, 0)
        with roborts_csm.Context(0) as c:
            c.set_outside_value(0.75)
            c.set_grid_stack(g, res, version=1)
            centers = np.array([[-20.0, 10.0, 0.3], [sx + 15.0, sy - 5.0, -1.0]])
            _, _, s1 = _check_same(c, f1["points"], p, np.arange(2), centers, max_depth=5)
            _, _, s2 = _check_same(c, f1["points"], p, np.arange(2), centers, max_depth=5, top_kernel=1)
            assert s1["top_box"] and not s2["top_box"] and s1["nodes"] == s2["nodes"]


@pytest.mark.parametrize("size,depth,penalty", [(2.0, 1, False), (2.0, 2, True), (2.0, 3, False), (2.0, 6, True),
                                                (2.35, 1, True), (2.5, 1, False), (2.75, 1, True), (3.15, 1, False),
                                                (0.8, 1, True), (1.95, 1, False), (1.5, 1, True), (0.3, 1, False),
                                                (2.2, 1, True)])
def test_top_boxes_equal_gathers(f1, stack5, size, depth, penalty):
    """The top level as beam boxes (pyr_topbox_kernel, every (pieces, loads)
    instantiation: nj = 21, 11, 6, 1, 24, 26, 28, 32, 9, 20, 16, 4, 23) writes the same
    bounds as the per-node gather kernel: the searches visit the same nodes
    at every level and return the exhaustive argmax."""
    import roborts_csm
    from roborts_csm.loop_closure import world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    res = float(f1["resolution"])
    p = CorrelationScanMatchParam(size, 0.05, 0.6, 0.0349, 0.5, 100, 0, penalty, 0)
    with roborts_csm.Context(0) as c:
        c.set_grid_stack(stack5, res, version=3)
        centers = np.stack([world_to_map(f1["init_pose"], res, f1["offset"])] * stack5.shape[0])
        centers[1, :2] += (17.0, -9.0)
        centers[3, :2] = (-3.0, 2.5)  # hanging off the grid's low corner
        gi = np.arange(stack5.shape[0])
        b1, w1, s1 = _check_same(c, f1["points"], p, gi, centers, max_depth=depth)
        b2, w2, s2 = c.search_windows(f1["points"], p, gi, centers, max_depth=depth, top_kernel=1)
        assert s1["top_box"] and not s2["top_box"]
        assert (w1, b1.score, b1.flat_index) == (w2, b2.score, b2.flat_index)
        assert s1["nodes"] == s2["nodes"] and s1["probe_leaves"] == s2["probe_leaves"]


@pytest.mark.parametrize("depth,penalty", [(1, False), (2, True), (3, False), (4, True)])
def test_search_long_scans(config3, depth, penalty):
    """Every beam of 1081-beam scans summed: the level passes split each node's
    beams over 8 lanes (pyr_bound_lanes) and, with one or two windows, the top
    level's beams over several waves per angle. Same answer as the exhaustive
    device argmax, at several depths, on three submaps and on one."""
    import roborts_csm
    from roborts_csm.loop_closure import world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    bases, batch = config3
    pts = batch.points_cells[batch.offsets[0]:batch.offsets[1]]
    assert pts.shape[0] >= 1024
    res = bases[0].resolution
    p = CorrelationScanMatchParam(3.0, 0.05, 0.8, 0.0349, 0.5, pts.shape[0], 0, penalty, 0)
    stack = np.stack([b.grid for b in bases])
    centers = np.stack([world_to_map(batch.init_poses[0], res, b.offset) for b in bases])
    with roborts_csm.Context(0) as c:
        c.set_grid_stack(stack, res, version=1)
        for gi in (np.arange(3), np.array([1])):
            _, _, st = _check_same(c, pts, p, gi, centers[gi], max_depth=depth)
            assert st["top_box"] and not st["exhaustive"]


def test_search_non_unit_step_is_exhaustive(f1, stack5):
    """A window step other than one cell is outside the pooled search: the
    call falls back to the exhaustive device search, same result."""
    import roborts_csm
    from roborts_csm.params import CorrelationScanMatchParam
    res = float(f1["resolution"])
    p = CorrelationScanMatchParam(1.0, 0.1, 0.3, 0.0349, 0.5, 100, 0, False, 0)
    with roborts_csm.Context(0) as c:
        c.set_grid_stack(stack5, res, version=3)
        centers = np.array([[150.0, 160.0, 0.0]] * stack5.shape[0])
        _, _, st = _check_same(c, f1["points"], p, np.arange(stack5.shape[0]), centers)
        assert st["exhaustive"]


@pytest.fixture(scope="module")
def config3():
    from roborts_csm import worlds
    side, res = 800, 0.05
    bases = [worlds.make_world(side, side, res, seed=20261015 + k) for k in range(3)]
    batch = worlds.make_scan_batch(bases[0], 1, seed=7)
    return bases, batch


def test_config3_real_window(config3):
    """BASELINE config 3 at its real size: +-8 m / +-pi, 181 x 321^2
    candidates per submap, B = 109, 3 submaps of 800 x 800 (the bench's
    submaps are shifted copies of such worlds). Search == exhaustive ==
    the oracle's whole-window argmax, submap by submap."""
    import roborts_csm
    from roborts_csm.loop_closure import world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    bases, batch = config3
    pts = batch.points_cells[batch.offsets[0]:batch.offsets[1]]
    pose = batch.init_poses[0]
    res = bases[0].resolution
    stack = np.stack([b.grid for b in bases])
    p = CorrelationScanMatchParam(16.0, 0.05, math.pi, 0.0349, 0.5, 100, 0, False, 0)
    na, ns = roborts_csm.window_dims(p)
    assert (na, ns) == (181, 321)
    centers = np.stack([world_to_map(pose, res, b.offset) for b in bases])
    with roborts_csm.Context(0) as c:
        c.set_grid_stack(stack, res, version=1)
        b, w, st = _check_same(c, pts, p, np.arange(3), centers)
        O.set_threads(16)
        try:
            got = [O.best_window(O.Map(bases[g].grid, res, bases[g].offset), pts, p, centers[g]) for g in range(3)]
        finally:
            O.set_threads(1)
        k, _ = _reduce(np.array([s for s, _ in got]), np.array([f for _, f in got]), na * ns * ns)
        assert w == k and b.score == got[k][0] and b.flat_index == got[k][1]
        assert st["beam_reads"] < st["candidates"] * 109 // 4  # the bound prunes most of the window


def test_config3_global_index_beyond_2_32(config3):
    """240 resident submaps; the only non-empty one is submap 233, so the
    winning global index (submap * 18,650,421 + flat) exceeds 2^32. The
    loop-closure shard reports it through both searches."""
    import roborts_csm
    from roborts_csm.loop_closure import ShardedLoopClosure, world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    bases, batch = config3
    pts = batch.points_cells[batch.offsets[0]:batch.offsets[1]]
    pose = batch.init_poses[0]
    res = bases[0].resolution
    n = 240
    stack = np.zeros((n,) + bases[0].grid.shape, dtype=np.float32)
    stack[233] = bases[0].grid
    offsets = np.tile(np.asarray(bases[0].offset), (n, 1))
    p = CorrelationScanMatchParam(16.0, 0.05, math.pi, 0.0349, 0.5, 100, 0, False, 0)
    na, ns = roborts_csm.window_dims(p)
    with roborts_csm.Context(0) as c:
        c.set_outside_value(0.0)
        c.set_grid_stack(stack, res, version=1)
        centers = np.stack([world_to_map(pose, res, o) for o in offsets])
        b, w, _ = c.search_windows(pts, p, np.arange(n), centers)
        assert w == 233
        gidx = 233 * na * ns * ns + b.flat_index
        assert gidx > 2 ** 32
        ex = ShardedLoopClosure(c, n, res, offsets, search="exhaustive").match(pts, p, pose)
        py = ShardedLoopClosure(c, n, res, offsets, search="pyramid").match(pts, p, pose)
        assert ex.global_index == py.global_index == gidx and ex.score == py.score == b.score
        assert ex.submap == py.submap == 233 and (ex.x, ex.y, ex.angle) == (py.x, py.y, py.angle)
        O.set_threads(16)
        try:
            m = O.Map(bases[0].grid, res, bases[0].offset, outside=0.0)
            s2, f2 = O.best_window(m, pts, p, centers[233])
        finally:
            O.set_threads(1)
        assert b.score == s2 and b.flat_index == f2


def test_config4_willow_20m():
    """BASELINE config 4: the willow map, the bench's 20 m / +-pi window
    (181 x 401^2 candidates), every beam summed; search == exhaustive ==
    oracle."""
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.loop_closure import world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    w = worlds.willow_world()
    batch = worlds.make_scan_batch(w, 1, seed=31)
    pts = batch.points_cells[batch.offsets[0]:batch.offsets[1]]
    p = CorrelationScanMatchParam(20.0, 0.05, math.pi, 0.0349, 0.5, 1081, 0, False, 0)
    center = world_to_map(batch.init_poses[0], w.resolution, w.offset)
    with roborts_csm.Context(0) as c:
        c.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 1))
        got = c.best_window(pts, p, center)
        b, win, st = c.search_windows(pts, p, [0], center.reshape(1, 3))
        assert win == 0 and b.score == got.score and b.flat_index == got.flat_index
        assert (b.x, b.y, b.angle) == (got.x, got.y, got.angle)
        # one window: the top level's beams are split over several waves per
        # angle, their sums added; the same answer and top level as the
        # per-node gathers (the levels below may differ: the probe roots are
        # the best of segments of each kernel's own block partials)
        b2, _, st2 = c.search_windows(pts, p, [0], center.reshape(1, 3), top_kernel=1)
        assert st["top_box"] and not st2["top_box"]
        assert st["nodes"][st["depth"]] == st2["nodes"][st2["depth"]]
        assert (b2.score, b2.flat_index) == (b.score, b.flat_index)
        O.set_threads(16)
        try:
            s2, f2 = O.best_window(O.Map(w.grid, w.resolution, w.offset), pts, p, center)
        finally:
            O.set_threads(1)
        assert b.score == s2 and b.flat_index == f2


def test_config4_willow_whole_map():
    """BASELINE config 4 as SURVEY 8d defines it: the whole padded willow map
    as the window (1566^2 cells around the map's centre x 181 angles = 444 M
    candidates), every beam summed. The admissible search equals the
    exhaustive argmax; the oracle (a whole-map oracle query is ~2 min of all
    cores, so not here) confirms the winner's score bit for bit by scoring
    that one candidate (a window of one position and one angle at the
    winner's pose: the same cell lattice, the same angle value, so the same
    host sincos); the exhaustive kernels are checked element-wise against the
    oracle on smaller windows in the tests above."""
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.loop_closure import world_to_map
    from roborts_csm.params import CorrelationScanMatchParam
    w = worlds.willow_world()
    sy, sx = w.grid.shape
    batch = worlds.make_scan_batch(w, 1, seed=31)
    pts = batch.points_cells[batch.offsets[0]:batch.offsets[1]]
    p = CorrelationScanMatchParam(max(sx, sy) * w.resolution, 0.05, math.pi, 0.0349, 0.5, 1081, 0, False, 0)
    na, ns = roborts_csm.window_dims(p)
    assert na == 181 and ns >= max(sx, sy)
    center = np.array([sx / 2.0, sy / 2.0, world_to_map(batch.init_poses[0], w.resolution, w.offset)[2]])
    with roborts_csm.Context(0) as c:
        c.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 1))
        got = c.best_window(pts, p, center)
        b, win, st = c.search_windows(pts, p, [0], center.reshape(1, 3))
        assert win == 0 and b.score == got.score and b.flat_index == got.flat_index
        assert (b.x, b.y, b.angle) == (got.x, got.y, got.angle)
        assert got.score > 0.5  # the scan found its place in the map
        one = CorrelationScanMatchParam(0.0, 0.05, 0.0, 0.0349, 0.5, 1081, 0, False, 0)
        assert roborts_csm.window_dims(one) == (1, 1)
        at = np.array([got.x, got.y, got.angle])
        g1 = c.best_window(pts, one, at)
    s1, f1 = O.best_window(O.Map(w.grid, w.resolution, w.offset), pts, one, at)
    assert f1 == 0 and s1 == got.score and g1.score == got.score
