"""The back-end scan-match service (include/csm_backend.h; SURVEY.md 8f row f2:
SlamProcessor::ScanMatchInterface slam/slam_processor.cpp:250-326, called by
RangeScanPoseGraph::LinkNearChains / TryCloseLoop).

CPU: the oracle's restatement recovers the query poses of a ray-cast drive.
GPU: a batch of jobs equals the oracle job by job bit for bit (pose,
covariance, score, map penalty, optimiser cost) and in the rebuilt maps —
batched over a stack of fine maps (both YAMLs: no optimiser), job by job
(optimiser on), and when a map grows (the batch falls back job by job).
"""
import numpy as np
import pytest

from roborts_csm import worlds

N_SCANS = 48


@pytest.fixture(scope="module")
def drive():
    w = worlds.make_world(400, 400, 0.05, seed=8)
    return w, worlds.make_scan_stream(w, N_SCANS, seed=9)


def _kept_poses(st):
    rng = np.random.default_rng(10)
    return st.true_poses + rng.normal(size=st.true_poses.shape) * [0.01, 0.01, 0.003]


def _jobs(st):
    """(query id, chain ids, initial pose): near-chain links, a sparse chain, a
    far chain (loop-closure shape)."""
    t = st.true_poses
    d = np.array([0.06, -0.04, 0.03])
    return [
        (47, list(range(36, 46)), t[47] + d),
        (40, list(range(20, 40, 2)), t[40] - d),
        (30, list(range(0, 11)), t[30] + 0.5 * d),
        (44, list(range(38, 44)), t[44] + np.array([-0.03, 0.05, -0.02])),
    ]


def _pub_maps(w, st, kept):
    """The same CountCell PubMap on both sides (oracle, device or None)."""
    import pyoracle as O
    o = O.GridMap(1, w.resolution, (w.size_x, w.size_y), w.offset, 0.0, 0.5)
    o.set_options(True, False, 0.72, 0.2)
    for k in range(N_SCANS):
        o.update_by_range(st.points_m[k] / w.resolution, kept[k])
    return o


def _device_pub(w, st, kept):
    from roborts_csm.gridmap import OccuGridMap
    m = OccuGridMap(w.resolution, (w.size_x, w.size_y), w.offset, 0.0, 0.5, kind=1)
    m.set_options(True, False, 0.72, 0.2)
    for k in range(N_SCANS):
        m.UpdateMapByRange(st.points_m[k] / w.resolution, kept[k])
    return m


def _param(mode):
    from roborts_csm.backend import BackEndParam
    from roborts_csm.params import PARAM_CONFIG_OPTIMIZE
    if mode == "sim":
        return BackEndParam()
    if mode == "opt":
        return BackEndParam(use_optimize_scan_match=True, optimize=PARAM_CONFIG_OPTIMIZE, optimize_failed_cost=20.0)
    if mode == "coarse_only":  # use_fine_scan_match = false path
        return BackEndParam()
    raise ValueError(mode)


def _oracle_run(prm, st, kept, jobs, cur, pub, use_fine=True):
    import pyoracle as O
    from roborts_csm.backend import job_results, make_jobs
    be = O.BackEnd(prm.to_c())
    for k in range(N_SCANS):
        assert be.add_scan(st.points_m[k], kept[k]) == k
    arr = make_jobs([st.points_m[q] for q, _, _ in jobs], [c for _, c, _ in jobs], [p for _, _, p in jobs],
                    use_fine)
    be.scan_match(arr, len(jobs), cur, pub)
    return be, job_results(arr, len(jobs))


def test_oracle_backend_recovers_query_poses(drive):
    w, st = drive
    kept = _kept_poses(st)
    pub = _pub_maps(w, st, kept)
    jobs = _jobs(st)
    _, res = _oracle_run(_param("sim"), st, kept, jobs, st.true_poses[-1], pub)
    for (q, _, _), r in zip(jobs, res):
        err = r.pose - st.true_poses[q]
        assert np.hypot(err[0], err[1]) < 0.03 and abs(err[2]) < 0.01, (q, err)
        assert 0.0 < r.score <= 1.0 and 0.0 < r.map_penalty <= 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sim", "opt", "coarse_only"])
def test_device_backend_matches_oracle(drive, mode):
    from map_engines import same_state
    from roborts_csm.backend import ScanMatchService
    w, st = drive
    kept = _kept_poses(st)
    jobs = _jobs(st)
    prm = _param(mode)
    use_fine = mode != "coarse_only"
    cur = st.true_poses[-1]
    obe, want = _oracle_run(prm, st, kept, jobs, cur, _pub_maps(w, st, kept), use_fine)
    svc = ScanMatchService(prm)
    for k in range(N_SCANS):
        assert svc.AddRangeData(st.points_m[k], kept[k]) == k
    pub = _device_pub(w, st, kept)
    got = svc.scan_match_jobs([st.points_m[q] for q, _, _ in jobs], [c for _, c, _ in jobs],
                              [p for _, _, p in jobs], cur, pub, use_fine)
    for j, (a, b) in enumerate(zip(want, got)):
        assert np.array_equal(a.pose, b.pose) and np.array_equal(a.cov, b.cov), (mode, j)
        assert (a.score, a.map_penalty, a.optimize_cost) == (b.score, b.map_penalty, b.optimize_cost), (mode, j)

    class _O:
        def __init__(self, m):
            self.m = m

        def state(self):
            i = self.m.info()
            return {"size_x": i["size_x"], "size_y": i["size_y"], "map_update_index": i["map_update_index"],
                    "cur_update_index": i["cur_update_index"], "offset": i["offset"], "bound": i["bound"]}

        def arrays(self):
            p, ps, h, u = self.m.cells()
            return p, ps, h, u, self.m.touched().reshape(p.shape)

    class _D(_O):
        def state(self):
            s = self.m.state()
            return {"size_x": s.size_x, "size_y": s.size_y, "map_update_index": s.map_update_index,
                    "cur_update_index": s.cur_update_index, "offset": (s.offset_x, s.offset_y),
                    "bound": (s.bound_min_x, s.bound_min_y, s.bound_max_x, s.bound_max_y)}

        def arrays(self):
            return self.m.cells()

    for slot in (0, len(jobs) - 1):
        for which in (0, 1):
            same_state(_O(obe.map(slot, which)), _D(svc.map(slot, which)))
    # a single job is one reference call on pair 0; it follows the batch's pair-0 history
    pose = np.array(jobs[0][2], dtype=np.float64)
    s1, cov1 = svc.ScanMatchInterface(st.points_m[jobs[0][0]], jobs[0][1], pose, cur, pub, use_fine)
    assert np.array_equal(pose, want[0].pose) and s1 == want[0].score and np.array_equal(cov1, want[0].cov)
    svc.close()


@pytest.mark.gpu
def test_device_backend_map_growth(drive):
    """Current pose far from a query: MapSizeCheck grows that job's maps, the
    batch falls back job by job, results still equal the oracle's."""
    from roborts_csm.backend import ScanMatchService
    w, st = drive
    kept = _kept_poses(st)
    jobs = _jobs(st)
    prm = _param("sim")
    cur = st.true_poses[30] + np.array([1.8, -1.7, 0.0])
    _, want = _oracle_run(prm, st, kept, jobs, cur, None)
    svc = ScanMatchService(prm)
    for k in range(N_SCANS):
        svc.AddRangeData(st.points_m[k], kept[k])
    got = svc.scan_match_jobs([st.points_m[q] for q, _, _ in jobs], [c for _, c, _ in jobs],
                              [p for _, _, p in jobs], cur, None)
    for a, b in zip(want, got):
        assert np.array_equal(a.pose, b.pose) and np.array_equal(a.cov, b.cov) and a.score == b.score
    sizes = {svc.map(j, 1).state().size_x for j in range(len(jobs))}
    assert len(sizes) > 1 and min(sizes) > 2400  # every pair grew, by different amounts
    svc.close()
