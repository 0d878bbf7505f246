"""GPU parity of the palette box kernel (csrc/csm_box.hip
score_box_pair_kernel v11, csrc/csm_palette.hip) against the CPU oracle.

The kernel reads one-cell-step windows (n_space <= 13: the coarse level of
every shipped parameter set, correlate_scan_matcher.h:552-584,637-662)
through the palette copy of the fixed-point grid: one byte per cell, the
index of the cell's value among the grid's distinct values. The bar is the
same as for every other kernel: all scores bit for bit, the argmax index
equal. Covered here: the palette's size limits (up to 16 values: the v11 pair
kernel over the strip copies, index shift 3 up to 8 values and 4 above; more:
the v6 box kernel reads gridi; CSM_KERNEL=v8 runs v6 for small palettes too,
the comparison), cells below the
outside value (negative fixed-point entries), windows off every edge, beams
on rounding boundaries, a grid stack (the palette grid's per-grid stride),
and the palette rebuilt after row and cell refreshes of a resident map.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import pyoracle as O  # noqa: E402


@pytest.fixture(scope="module")
def f1(golden_dir):
    return np.load(os.path.join(golden_dir, "f1_config1.npz"))


def _level(n_points):
    from roborts_csm.params import SIM_YAML_LEVELS
    lv = SIM_YAML_LEVELS[0]  # 0.6 m at 0.05 m on a 0.05 m map: 13 x 13, one-cell steps
    return lv.with_(use_point_size=int(n_points))


def _points(f1):
    extra = np.array([[0.0, 0.0], [0.0, 0.0], [1.0, -2.0], [-300.0, 3.0], [2.0, -300.0], [250.0, 250.0],
                      [0.25, 0.0]])
    return np.ascontiguousarray(np.concatenate([f1["points"], extra]))


def _centers(res, size=0.6):
    half = (size / res) * 0.5
    return [np.array(c) for c in ([100.5 + half, 200.5 + half, 0.0], [100.5 + half, 200.5 + half, 1.3],
                                  [200.0 + 3 * 2.0 ** -43, 199.0 + 2.0 ** -43, 0.7], [3.2, 2.1, -2.5],
                                  [396.0, 398.0, 1.0], [255.0 + 2.0 ** -44, 130.3, 3.0])]


def _ctx(**env):
    """A context whose single-window calls take the throughput kernels
    (CSM_SMALL=0: not the few-window split kernel)."""
    import roborts_csm
    env = dict({"CSM_SMALL": "0"}, **env)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c = roborts_csm.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    c.set_profiling(True)
    return c


def _check_windows(c, m, pts, lv, centers):
    for cen in centers:
        want = O.score_window(m, pts, lv, cen, 30 * 13 * 13)
        assert np.array_equal(c.score_window(pts, lv, cen), want), cen
        got = c.best_window(pts, lv, cen)
        s, flat = O.best_window(m, pts, lv, cen)
        assert got.score == s and got.flat_index == flat, cen


def _stats(c):
    return {k["name"]: k for k in c.kernel_stats()}


def _kernel(grids, outside=0.3, pair=True):
    """The box kernel the palette of `grids` selects: its size is the number
    of distinct values other than the outside value, plus the outside value."""
    g = np.asarray(grids, dtype=np.float32)
    n = len(np.unique(g[g != np.float32(outside)])) + 1
    return "score_box_pair_kernel" if (pair and n <= 16) else "score_box_kernel"


def _values(n, rng, lo=0.3125, step=2.0 ** -12):
    """n distinct float32 values, all multiples of 2^-12 (exactly summable)."""
    v = lo + step * np.arange(n, dtype=np.float64)
    return rng.permutation(v).astype(np.float32)


@pytest.mark.parametrize("n_values,kernel", [(256, "score_box_kernel"), (257, "score_box_kernel"),
                                            (2, "score_box_pair_kernel"), (8, "score_box_pair_kernel"),
                                            (9, "score_box_pair_kernel"), (16, "score_box_pair_kernel"),
                                            (17, "score_box_kernel")])
def test_palette_size_limits(f1, n_values, kernel):
    """The outside value plus n_values - 1 others: up to 16 values take the
    pair kernel (pair codes of 3 bits per index up to 8 values, 4 above),
    more the v6 box kernel over gridi; all bit-exact."""
    import roborts_csm
    rng = np.random.default_rng(n_values)
    res = float(f1["resolution"])
    vals = np.concatenate([[np.float32(0.3)], _values(n_values - 1, rng)])
    g = rng.choice(vals, size=f1["grid"].shape).astype(np.float32)
    g.ravel()[:n_values] = vals  # every value present
    m = O.Map(g, res, tuple(f1["offset"]))
    pts = _points(f1)
    lv = _level(pts.shape[0])
    c = _ctx()
    try:
        c.set_grid(roborts_csm.ScanMatchMap(g, res, tuple(f1["offset"]), 0, 1))
        _check_windows(c, m, pts, lv, _centers(res))
        st = _stats(c)
        assert kernel + "<13,all>" in st and kernel + "<13,best>" in st, st.keys()
        assert len([k for k in st if k.startswith("score_box")]) == 2, st.keys()
        if n_values <= 256:
            assert st["grid:palette"]["scorings"] == n_values
    finally:
        c.close()


@pytest.mark.parametrize("pair", [True, False])
def test_palette_negative_values_and_blur(f1, pair):
    """The reference's blurred map (f1) with some cells below the outside
    value (negative fixed-point entries) and an outside value of 0.5."""
    import roborts_csm
    res = float(f1["resolution"])
    g = np.array(f1["grid"], dtype=np.float32)
    rng = np.random.default_rng(5)
    g[rng.random(g.shape) < 0.05] = np.float32(0.0)
    g[rng.random(g.shape) < 0.02] = np.float32(0.125)
    pts = _points(f1)
    lv = _level(pts.shape[0])
    for outside in (0.3, 0.5):
        c = _ctx(**({} if pair else {"CSM_KERNEL": "v8"}))
        try:
            c.set_outside_value(outside)
            mo = O.Map(g, res, tuple(f1["offset"]), outside=outside)
            c.set_grid(roborts_csm.ScanMatchMap(g, res, tuple(f1["offset"]), 0, 1))
            _check_windows(c, mo, pts, lv, _centers(res))
            assert _kernel(g, outside, pair) + "<13,all>" in _stats(c)
        finally:
            c.close()


@pytest.mark.parametrize("pair", [True, False])
def test_palette_grid_stack(f1, pair):
    """best_windows over a stack of three grids with different palettes in
    one palette copy (grid_index > 0 reads at its own stride)."""
    res = float(f1["resolution"])
    rng = np.random.default_rng(11)
    base = np.array(f1["grid"], dtype=np.float32)
    stack = np.stack([base, np.roll(base, 37, axis=0),
                      rng.choice(np.array([0.3, 0.5, 0.75, 1.0], dtype=np.float32), size=base.shape)])
    pts = _points(f1)
    lv = _level(pts.shape[0])
    cen = np.stack(_centers(res))
    gi = np.array([0, 1, 2, 1, 2, 0], dtype=np.int32)
    c = _ctx(**({} if pair else {"CSM_KERNEL": "v8"}))
    try:
        c.set_grid_stack(stack, res, version=1)
        sc, flat, x, y, a = c.best_windows(pts, lv, gi, cen)
        for i in range(len(gi)):
            s, fl = O.best_window(O.Map(stack[gi[i]], res, (0.0, 0.0)), pts, lv, cen[i])
            assert sc[i] == s and flat[i] == fl, i
        assert _kernel(stack, 0.3, pair) + "<13,best>" in _stats(c)
    finally:
        c.close()


@pytest.mark.parametrize("pair", [True, False])
def test_palette_follows_grid_refresh(f1, pair):
    """A resident map refreshed by rows and by cells, with values the palette
    had not seen: the palette is rebuilt and the scores stay exact."""
    import roborts_csm
    res = float(f1["resolution"])
    g = np.array(f1["grid"], dtype=np.float32)
    mm = roborts_csm.ScanMatchMap(g, res, tuple(f1["offset"]), 0, 1)
    pts = _points(f1)
    lv = _level(pts.shape[0])
    cen = _centers(res)[:3]
    c = _ctx(**({} if pair else {"CSM_KERNEL": "v8"}))
    try:
        c.set_grid(mm)
        _check_windows(c, O.Map(g, res, tuple(f1["offset"])), pts, lv, cen)
        g[150:170, :] = np.float32(0.8125)
        mm.version = 2
        c.update_grid_rows(mm, 150, 170)
        _check_windows(c, O.Map(g, res, tuple(f1["offset"])), pts, lv, cen)
        idx = np.arange(200 * 400 + 100, 200 * 400 + 180, dtype=np.int32)
        g.ravel()[idx] = np.float32(0.6875)
        mm.version = 3
        c.update_grid_cells(mm, idx)
        _check_windows(c, O.Map(g, res, tuple(f1["offset"])), pts, lv, cen)
        st = _stats(c)
        if pair:  # (the v6 kernel reads gridi: no palette is built)
            assert st["grid:palette"]["launches"] >= 3
        assert _kernel(g, 0.3, pair) + "<13,all>" in st, st.keys()
    finally:
        c.close()


@pytest.mark.parametrize("pair", [True, False])
def test_palette_low_edge_straddle(f1, pair):
    """Windows whose boxes straddle the grid's low edges: the reference
    truncates toward zero, so a cell coordinate in (-1, 0) reads row / column
    0 and one at or below -1 the outside value. The pair kernel reads such
    beams from the strips' low-side padding (column -1 repeating column 0,
    row -1 repeating row 0); row 0 and column 0 hold values found nowhere else,
    so a padding that repeated the wrong cells would change the scores."""
    import roborts_csm
    res = float(f1["resolution"])
    rng = np.random.default_rng(23)
    vals = np.array([0.3, 0.375, 0.5, 0.625, 0.75, 0.875, 1.0], dtype=np.float32)
    g = rng.choice(vals[:5], size=f1["grid"].shape).astype(np.float32)
    g[0, :] = vals[5]
    g[:, 0] = vals[6]
    g[0, 0] = np.float32(0.4375)
    m = O.Map(g, res, tuple(f1["offset"]))
    # beam endpoints a few cells around the pose (boxes of 13 x 13 around them)
    pts = np.ascontiguousarray(rng.uniform(-14.0, 14.0, size=(700, 2)))
    pts[:40] = np.round(pts[:40] * 4.0) / 4.0  # quarter cells: corners on x0 + 0.5 + k / 4
    lv = _level(pts.shape[0])
    cens = []
    for i in range(12):
        x = rng.uniform(-8.0, 14.0) if i % 3 else rng.uniform(150.0, 250.0)
        y = rng.uniform(-8.0, 14.0) if i % 3 != 1 else rng.uniform(150.0, 250.0)
        cens.append(np.array([x, y, rng.uniform(-np.pi, np.pi)]))
    cens.append(np.array([6.0, 6.0, 0.0]))  # t on half cells: x0 + 0.5 integral
    c = _ctx(**({} if pair else {"CSM_KERNEL": "v8"}))
    try:
        c.set_grid(roborts_csm.ScanMatchMap(g, res, tuple(f1["offset"]), 0, 1))
        _check_windows(c, m, pts, lv, cens)
        assert _kernel(g, 0.3, pair) + "<13,all>" in _stats(c)
    finally:
        c.close()
