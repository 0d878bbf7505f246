"""GPU: incremental refresh and multi-map residency of host grids
(csm_update_grid_cells / csm_update_grid_rows / csm_set_grid slots).

The reference rewrites only the cells UpdateMapByRange touches
(occu_grid_map.h:258-329, map_update_point_ :509,528,571) and resets only
those in ResetValueSpeedup (grid_map_base.h:114-120); the device copy is
refreshed the same way. Every check compares a full 3-level match on the
mutated map with the oracle on the same host map, bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import pyoracle as O  # noqa: E402

CELL = np.dtype([("prob_value_", "<f4"), ("update_index_", "<i4")])


def _aos(grid):
    a = np.empty(grid.shape, dtype=CELL)
    a["prob_value_"] = grid
    a["update_index_"] = -1
    return a


@pytest.fixture(scope="module")
def scene():
    from roborts_csm import worlds
    w = worlds.make_world(600, 600, 0.05, seed=20261015)
    b = worlds.make_scan_batch(w, 6, seed=9)
    return w, b


def _levels():
    from roborts_csm.params import headline_levels
    return headline_levels()


def _check_match(ctx, w, b, cells, k):
    import roborts_csm
    pts = b.points_cells[b.offsets[k]:b.offsets[k + 1]]
    pose = b.init_poses[k].copy()
    cov = np.eye(3).reshape(9).copy()
    s = ctx.scan_matchers(pts, _levels(), pose, cov)
    om = O.Map(np.ascontiguousarray(cells["prob_value_"]), w.resolution, w.offset)
    s2, p2, c2 = O.scan_matchers(om, pts, _levels(), b.init_poses[k], np.eye(3))
    assert s == s2 and np.array_equal(pose, p2) and np.array_equal(cov, c2), k
    return roborts_csm


def _mutate(rng, cells, n, values):
    idx = rng.choice(cells.size, size=n, replace=False).astype(np.int32)
    flat = cells.reshape(-1)
    flat["prob_value_"][idx] = rng.choice(values, size=n).astype(np.float32)
    return idx


def test_update_cells_and_rows_exact(scene):
    import roborts_csm
    w, b = scene
    cells = _aos(w.grid)
    m = roborts_csm.ScanMatchMap(cells, w.resolution, w.offset, 0, 1)
    rng = np.random.default_rng(5)
    vals = np.unique(w.grid)
    with roborts_csm.Context(0) as ctx:
        ctx.set_profiling(True)
        ctx.set_grid(m)
        _check_match(ctx, w, b, cells, 0)
        for k in range(1, 4):
            idx = _mutate(rng, cells, 20000, vals)
            m.version += 1
            ctx.update_grid_cells(m, np.concatenate([idx, idx[:100]]))  # duplicates allowed
            _check_match(ctx, w, b, cells, k)
        # rows: rewrite a band of rows with other map values
        cells["prob_value_"][100:260] = np.roll(w.grid, 7, axis=1)[100:260]
        m.version += 1
        ctx.update_grid_rows(m, 100, 260)
        _check_match(ctx, w, b, cells, 4)
        st = {s["name"]: s for s in ctx.kernel_stats()}
        assert st["grid:upload"]["launches"] == 1  # only the first set_grid uploads the whole grid
        assert st["grid:cells"]["launches"] == 3 and st["grid:rows"]["launches"] == 1


def test_update_breaking_fixed_point_stays_exact(scene):
    """A value finer than the fixed-point granularity (or out of its range)
    forces the exact copy to be rebuilt before the next match."""
    import roborts_csm
    w, b = scene
    cells = _aos(w.grid)
    m = roborts_csm.ScanMatchMap(cells, w.resolution, w.offset, 0, 1)
    with roborts_csm.Context(0) as ctx:
        ctx.set_grid(m)
        _check_match(ctx, w, b, cells, 0)
        flat = cells.reshape(-1)
        idx = np.arange(1000, 200000, 97, dtype=np.int32)
        flat["prob_value_"][idx] = np.float32(0.3) + np.float32(2.0 ** -40)  # not a multiple of 2^-25
        m.version += 1
        ctx.update_grid_cells(m, idx)
        _check_match(ctx, w, b, cells, 1)
        flat["prob_value_"][idx[:10]] = np.float32(3.0e3)  # outside the int32 range at E = 25
        m.version += 1
        ctx.update_grid_cells(m, idx[:10])
        _check_match(ctx, w, b, cells, 2)


def test_maps_stay_resident_across_switches(scene):
    """Front-end fine map and back-end maps alternate on one context: each is
    uploaded once and stays resident (4 slots, LRU)."""
    import roborts_csm
    w, b = scene
    maps, host = [], []
    for s in range(4):
        g = np.roll(w.grid, 13 * s, axis=0)
        cells = _aos(g)
        host.append(cells)
        maps.append(roborts_csm.ScanMatchMap(cells, w.resolution, w.offset, 0, 1))
    with roborts_csm.Context(0) as ctx:
        ctx.set_profiling(True)
        for rnd in range(3):
            for s in range(4):
                ctx.set_grid(maps[s])
                _check_match(ctx, w, b, host[s], (rnd + s) % 6)
        st = {s["name"]: s for s in ctx.kernel_stats()}
        assert st["grid:upload"]["launches"] == 4
        # a fifth map evicts the least recently used (map 0): it is uploaded again
        extra = _aos(np.roll(w.grid, 5, axis=1))
        ctx.set_grid(roborts_csm.ScanMatchMap(extra, w.resolution, w.offset, 0, 1))
        _check_match(ctx, w, b, extra, 0)
        ctx.set_grid(maps[1])
        _check_match(ctx, w, b, host[1], 1)
        ctx.set_grid(maps[0])
        _check_match(ctx, w, b, host[0], 2)
        st = {s["name"]: s for s in ctx.kernel_stats()}
        assert st["grid:upload"]["launches"] == 6


def test_geometry_change_uploads_whole_grid(scene):
    """ExtendSize reallocates and resizes (grid_map_base.h:186-254): an update
    call with a new geometry falls back to a whole-grid upload."""
    import roborts_csm
    w, b = scene
    cells = _aos(w.grid)
    m = roborts_csm.ScanMatchMap(cells, w.resolution, w.offset, 0, 1)
    with roborts_csm.Context(0) as ctx:
        ctx.set_grid(m)
        big = np.full((700, 700), np.float32(0.3), dtype=np.float32)
        big[50:650, 50:650] = w.grid
        cells2 = _aos(big)
        off2 = (w.offset[0] + 50 * w.resolution, w.offset[1] + 50 * w.resolution)
        m2 = roborts_csm.ScanMatchMap(cells2, w.resolution, off2, 0, 2)
        ctx.update_grid_cells(m2, np.array([0, 1, 2], dtype=np.int32))
        pts = b.points_cells[b.offsets[0]:b.offsets[1]]
        pose = b.init_poses[0].copy()
        cov = np.eye(3).reshape(9).copy()
        s = ctx.scan_matchers(pts, _levels(), pose, cov)
        om = O.Map(big, w.resolution, off2)
        s2, p2, c2 = O.scan_matchers(om, pts, _levels(), b.init_poses[0], np.eye(3))
        assert s == s2 and np.array_equal(pose, p2) and np.array_equal(cov, c2)
