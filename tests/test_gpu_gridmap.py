"""GPU parity of the device-resident occupancy maps (SURVEY.md 8f rows f1,
f4; include/csm_gridmap.h) against the oracle (oracle/map_oracle.cpp), which
the CPU tests pin to an independent restatement. Bar: bit-identical cells
(prob / pass / hit / update_index), touched-cell set, geometry after growth,
update counters and map-check penalties — tolerance 0."""
import math

import numpy as np
import pytest

import map_scenarios as S
from map_engines import DeviceEngine, OracleEngine, same_state

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scans():
    return S.make_scans(4)


@pytest.mark.parametrize("name", sorted(S.scenarios()))
def test_device_map_matches_oracle(name, scans):
    sc = S.scenarios()[name]
    a, pa = S.run(OracleEngine, sc, *scans)
    b, pb = S.run(DeviceEngine, sc, *scans)
    same_state(a, b)
    assert pa == pb


def test_unsupported_modes_fail_loudly(scans):
    from roborts_csm.gridmap import COUNT_CELL, GridMapError, OccuGridMap
    pts, poses = scans
    m = OccuGridMap(0.05, (200, 200), (5.0, 5.0), 0.15, 0.3)
    m.set_options(True, False, 0.88, 0.2)  # full update + blur: order-dependent, unused by the reference
    with pytest.raises(GridMapError):
        m.UpdateMapByRange(pts[0], poses[0], use_blur=True)
    c = OccuGridMap(0.05, (200, 200), (5.0, 5.0), 0.15, 0.5, kind=COUNT_CELL)
    c.set_options(True, True, 0.88, 0.2)
    with pytest.raises(GridMapError):
        c.UpdateMapByRange(pts[0], poses[0], use_blur=True)


def _fine_map_stream(n_scans, seed=11):
    """1081-beam scans along a path, in 1 cm cells (fine_map_resolution 0.01)."""
    from roborts_csm import worlds
    w = worlds.make_world(400, 400, 0.05, seed=seed)
    laser = worlds.LaserSpec()
    rng = np.random.default_rng(seed)
    p0 = worlds.sample_free_poses(w, 1, rng, clearance_m=1.0)[0]
    poses = np.array([[p0[0] + 0.1 * k * math.cos(p0[2]), p0[1] + 0.1 * k * math.sin(p0[2]),
                       p0[2] + 0.02 * k] for k in range(n_scans)])
    rngs = worlds.raycast_ranges(w, poses, laser)
    return [worlds.scan_points(rngs[k], laser) * (1 / 0.01) for k in range(n_scans)], poses


def test_fine_scan_match_map_full_size():
    """Front-end fine ScanMatchMap as CreateAllMap builds it (slam_processor.cpp:
    466-510: 3*range_max at 0.01 m = 3000 x 3000 cells, sigma 0.03, offset 0.88,
    auto-resize, just_update_occu) fed a scan stream, then the back-end reset
    path (ResetScanMatchMapWithRangeVec :448-462)."""
    scans, poses = _fine_map_stream(6)
    sc = dict(kind=0, res=0.01, size=(3000, 3000), off=None, dev=0.03, default=0.3,
              opts=(True, True, 0.88, 0.2), cell=None, ops=[("update", k, True) for k in range(4)]
              + [("opts", (False, True, 0.88, 0.2)), ("offset", "shift"), ("init", [3, 4, 5], True, True)])
    sc["off"] = "centre"
    a, _ = S.run(OracleEngine, sc, scans, poses)
    b, _ = S.run(DeviceEngine, sc, scans, poses)
    same_state(a, b)


def test_matcher_reads_device_map():
    """csm_set_grid_gridmap: the 3-level match on the device map equals the
    oracle's match on the same cells."""
    import pyoracle as O
    import roborts_csm
    from roborts_csm.gridmap import OccuGridMap, set_matcher_grid
    from roborts_csm.params import SIM_YAML_LEVELS
    scans, poses = _fine_map_stream(4)
    res = 0.01
    off = (-(poses[0][0] - 0.5 * 1500 * res), -(poses[0][1] - 0.5 * 1500 * res))
    m = OccuGridMap(res, (1500, 1500), off, 0.03, 0.3)
    m.set_options(True, True, 0.88, 0.2)
    drawn = [m.UpdateMapByRange(scans[k], poses[k], use_blur=True) for k in range(3)]
    assert any(drawn)  # a scan that makes the map grow is not drawn (occu_grid_map.h:294-298)
    st = m.state()
    prob = m.cells()[0]
    init = poses[3] + np.array([0.03, -0.02, 0.02])
    with roborts_csm.Context(0) as ctx:
        set_matcher_grid(ctx, m)
        pose = init.copy()
        cov = np.eye(3).reshape(9).copy()
        s = ctx.scan_matchers(scans[3], SIM_YAML_LEVELS, pose, cov)
    om = O.Map(prob, st.resolution, (st.offset_x, st.offset_y), st.map_update_index)
    s2, pose2, cov2 = O.scan_matchers(om, scans[3], SIM_YAML_LEVELS, init, np.eye(3))
    assert s == s2 and np.array_equal(pose, pose2) and np.array_equal(cov, cov2)


def test_map_update_after_set_grid_is_ordered():
    """csm_set_grid_gridmap borrows the cells until the next set_grid; a map
    update issued right after it (no match in between) must wait for the
    matcher's reads: the match sees the cells as they were when the update was
    issued after the match was enqueued, so here (update after the match call
    returns) the matcher result is the oracle's on the pre-update cells, and a
    second match after the update sees the updated cells."""
    import pyoracle as O
    import roborts_csm
    from roborts_csm.gridmap import OccuGridMap, set_matcher_grid
    from roborts_csm.params import SIM_YAML_LEVELS
    scans, poses = _fine_map_stream(6)
    res = 0.01
    off = (-(poses[0][0] - 0.5 * 1500 * res), -(poses[0][1] - 0.5 * 1500 * res))
    m = OccuGridMap(res, (1500, 1500), off, 0.03, 0.3)
    m.set_options(True, True, 0.88, 0.2)
    for k in range(3):
        m.UpdateMapByRange(scans[k], poses[k], use_blur=True)
    with roborts_csm.Context(0) as ctx:
        for k in (3, 4):
            st = m.state()
            prob = m.cells()[0].copy()
            set_matcher_grid(ctx, m)
            init = poses[k] + np.array([0.03, -0.02, 0.02])
            pose = init.copy()
            cov = np.eye(3).reshape(9).copy()
            s = ctx.scan_matchers(scans[k], SIM_YAML_LEVELS, pose, cov)
            m.UpdateMapByRange(scans[k], poses[k], use_blur=True)  # right after: ordered after the reads
            om = O.Map(prob, st.resolution, (st.offset_x, st.offset_y), st.map_update_index)
            s2, pose2, cov2 = O.scan_matchers(om, scans[k], SIM_YAML_LEVELS, init, np.eye(3))
            assert s == s2 and np.array_equal(pose, pose2) and np.array_equal(cov, cov2), k


def test_matcher_uses_map_mirror_exactly():
    """The map keeps a fixed-point mirror of its cells (every kernel that
    writes prob writes it too), so csm_set_grid_gridmap no longer analyses and
    converts the whole grid per scan. Through blur updates, a growth, a blur
    offset change (new splat values), the back end's reset speed-up and a
    full reset, every borrow uses the mirror and every score of three windows
    equals the oracle's on the downloaded cells; a map that took a line update
    (device-computed values) falls back to the whole-grid conversion, still
    exact."""
    import pyoracle as O
    import roborts_csm
    from roborts_csm.gridmap import OccuGridMap, set_matcher_grid
    from roborts_csm.params import SIM_YAML_LEVELS
    scans, poses = _fine_map_stream(8)
    res = 0.01
    off = (-(poses[0][0] - 0.5 * 700 * res), -(poses[0][1] - 0.5 * 700 * res))

    def check(ctx, m, k, want_mirror):
        ctx.set_profiling(True)
        set_matcher_grid(ctx, m)
        st = m.state()
        prob = m.cells()[0]
        om = O.Map(prob, st.resolution, (st.offset_x, st.offset_y), st.map_update_index)
        c = O.world_to_map(om, poses[k] + np.array([0.02, -0.01, 0.01]))
        for lv in SIM_YAML_LEVELS:
            got = ctx.score_window(scans[k], lv, c)
            assert np.array_equal(got, O.score_window(om, scans[k], lv, c, got.size)), (k, lv)
        names = {s["name"] for s in ctx.kernel_stats()}
        ctx.set_profiling(False)
        assert ("grid:mirror" in names) == want_mirror and ("grid:analyze" in names) != want_mirror, names

    with roborts_csm.Context(0) as ctx:
        m = OccuGridMap(res, (700, 700), off, 0.03, 0.3)
        m.set_options(True, True, 0.88, 0.2)
        for k in range(3):  # blur splats; the 700-cell map grows under the 10 m scans
            m.UpdateMapByRange(scans[k], poses[k], use_blur=True)
            check(ctx, m, k + 1, True)
        m.set_options(True, True, 0.72, 0.2)  # new splat values
        m.UpdateMapByRange(scans[4], poses[4], use_blur=True)
        check(ctx, m, 5, True)
        m.InitMapWithRangeVec([scans[5], scans[6]], [poses[5], poses[6]], use_blur=True, use_reset_speedup=True)
        check(ctx, m, 7, True)
        m.Reset()
        check(ctx, m, 7, True)
        lines = OccuGridMap(res, (700, 700), off, 0.0, 0.3)
        lines.set_options(True, False, 0.88, 0.2)
        drawn = [lines.UpdateMapByRange(scans[k], poses[k]) for k in range(3)]  # the first grows the map
        assert any(drawn)
        check(ctx, lines, 3, False)
