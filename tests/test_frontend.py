"""The online front-end (include/csm_frontend.h; SlamProcessor::process,
slam/slam_processor.cpp:65-248; BASELINE config 5).

CPU: the oracle's restatement of the loop tracks a ray-cast drive.
GPU: the device front-end equals the oracle scan by scan (pose, matched pose,
covariance, score, map penalty, gates) and in its three maps — bit for bit."""
import math

import numpy as np
import pytest

from roborts_csm import worlds


def _stream(n, seed=3):
    w = worlds.make_world(400, 400, 0.05, seed=seed)
    return worlds.make_scan_stream(w, n, seed=seed)


def _rel(true, k):
    d = true[k] - true[0]
    c, s = math.cos(-true[0, 2]), math.sin(-true[0, 2])
    return np.array([c * d[0] - s * d[1], s * d[0] + c * d[1], d[2]])


def _param(mode):
    """sim: simulatin_param.yaml (no optimizer); opt_sim: with the Gauss-Newton
    matcher and the YAML's optimize_failed_cost 2 (often falls back to the
    correlative coarse level); opt_mixed: failed cost 0.33, so some scans take
    the fallback and some do not; opt_cfg: ParamConfig's optimizer defaults
    (failed cost 20: the optimizer replaces the coarse level)."""
    from roborts_csm.frontend import FrontEndParam
    from roborts_csm.params import PARAM_CONFIG_OPTIMIZE, PARAM_CONFIG_OPTIMIZE_FAILED_COST
    if mode == "sim":
        return FrontEndParam()
    if mode == "opt_sim":
        return FrontEndParam(use_optimize_scan_match=True)
    if mode == "opt_mixed":  # failed cost inside the drive's cost range: both branches of :224
        return FrontEndParam(use_optimize_scan_match=True, optimize_failed_cost=0.33)
    return FrontEndParam(use_optimize_scan_match=True, optimize=PARAM_CONFIG_OPTIMIZE,
                         optimize_failed_cost=PARAM_CONFIG_OPTIMIZE_FAILED_COST)


@pytest.mark.parametrize("mode", ["sim", "opt_sim", "opt_mixed", "opt_cfg"])
def test_oracle_frontend_tracks_drive(mode):
    import pyoracle as O
    from roborts_csm.frontend import CsmFrontendResult
    st = _stream(30)
    fe = O.FrontEnd(_param(mode).to_c())
    for k in range(30):
        r = fe.process(st.points_m[k], st.odom_poses[k], CsmFrontendResult())
        err = np.array(r.pose[:]) - _rel(st.true_poses, k)
        assert abs(err[0]) < 0.02 and abs(err[1]) < 0.02 and abs(err[2]) < 0.01, (k, err)
        assert r.map_updated


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sim", "opt_sim", "opt_mixed", "opt_cfg"])
def test_device_frontend_matches_oracle(mode):
    import pyoracle as O
    from roborts_csm.frontend import CsmFrontendResult, SlamFrontEnd
    n = 24
    st = _stream(n, seed=4)
    prm = _param(mode)
    ofe = O.FrontEnd(prm.to_c())
    dfe = SlamFrontEnd(prm)
    for k in range(n):
        a = ofe.process(st.points_m[k], st.odom_poses[k], CsmFrontendResult())
        b = dfe.process(st.points_m[k], st.odom_poses[k])
        assert np.array_equal(np.array(a.pose[:]), b.pose), k
        assert np.array_equal(np.array(a.match_pose[:]), b.match_pose), k
        assert np.array_equal(np.array(a.cov[:]), b.cov), k
        assert (a.score, a.map_penalty, a.optimize_cost, a.data_index, bool(a.map_updated),
                bool(a.pose_accepted)) == \
            (b.score, b.map_penalty, b.optimize_cost, b.data_index, b.map_updated, b.pose_accepted), k

    _same_maps(ofe, dfe)
    dfe.close()


def _same_maps(ofe, dfe):
    from map_engines import same_state

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

    class _D:
        def __init__(self, m):
            self.m = m

        def state(self):
            s = self.m.state()
            return {"size_x": s.size_x, "size_y": s.size_y, "map_update_index": s.map_update_index,
                    "cur_update_index": s.cur_update_index, "offset": (s.offset_x, s.offset_y),
                    "bound": (s.bound_min_x, s.bound_min_y, s.bound_max_x, s.bound_max_y)}

        def arrays(self):
            return self.m.cells()

    for which in (0, 1, 2):
        same_state(_O(ofe.map(which)), _D(dfe.map(which)))


def _corrections(kept, k_ids=(1, 4, 9, 13)):
    """A pose-graph style correction: some kept scans move a few cm / mrad."""
    rng = np.random.default_rng(17)
    ids = np.array([i for i in k_ids if i < kept.shape[0]], dtype=np.int32)
    poses = kept[ids] + rng.uniform(-1, 1, size=(ids.size, 3)) * np.array([0.04, 0.04, 0.01])
    return ids, poses


def test_oracle_correct_pose_and_map():
    """CPU: the oracle's CorrectPoseAndMap (slam_processor.cpp:329-370)
    rebuilds its maps and the loop keeps tracking; a bad id is refused."""
    import pyoracle as O
    from roborts_csm.frontend import CsmFrontendResult
    st = _stream(26, seed=5)
    fe = O.FrontEnd(_param("sim").to_c())
    for k in range(20):
        fe.process(st.points_m[k], st.odom_poses[k], CsmFrontendResult())
    with pytest.raises(ValueError):
        fe.correct_pose_and_map([99], [[0.0, 0.0, 0.0]])
    fe.correct_pose_and_map([2, 5], [[0.01, 0.0, 0.0], [0.0, 0.02, 0.005]])
    for k in range(20, 26):
        r = fe.process(st.points_m[k], st.odom_poses[k], CsmFrontendResult())
        err = np.array(r.pose[:]) - _rel(st.true_poses, k)
        assert abs(err[0]) < 0.05 and abs(err[1]) < 0.05 and abs(err[2]) < 0.02, (k, err)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sim", "opt_sim"])
def test_device_correct_pose_and_map_matches_oracle(mode):
    """SlamProcessor::CorrectPoseAndMap on the device: corrected poses, the
    three maps rebuilt from every kept scan (PubMap with the passthrough
    copies of scan 0, blurred scan-match maps), bit for bit against the
    oracle; then the front-end runs on over the rebuilt maps, still equal."""
    import pyoracle as O
    from roborts_csm.frontend import CsmFrontendResult, SlamFrontEnd
    st = _stream(30, seed=6)
    prm = _param(mode)
    ofe = O.FrontEnd(prm.to_c())
    dfe = SlamFrontEnd(prm)
    try:
        for k in range(22):
            ofe.process(st.points_m[k], st.odom_poses[k], CsmFrontendResult())
            dfe.process(st.points_m[k], st.odom_poses[k])
        kept = dfe.kept_poses()
        assert kept.shape[0] >= 10
        ids, poses = _corrections(kept)
        ofe.correct_pose_and_map(ids, poses)
        dfe.correct_pose_and_map(ids, poses)
        assert np.array_equal(dfe.kept_poses()[ids], poses)
        _same_maps(ofe, dfe)
        for k in range(22, 30):
            a = ofe.process(st.points_m[k], st.odom_poses[k], CsmFrontendResult())
            b = dfe.process(st.points_m[k], st.odom_poses[k])
            assert np.array_equal(np.array(a.pose[:]), b.pose), k
            assert (a.score, a.map_penalty, bool(a.map_updated)) == (b.score, b.map_penalty, b.map_updated), k
        _same_maps(ofe, dfe)
        with pytest.raises(RuntimeError):
            dfe.correct_pose_and_map([10 ** 6], [[0.0, 0.0, 0.0]])
    finally:
        dfe.close()
