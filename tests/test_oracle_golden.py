"""CPU: the oracle against the committed golden vectors, and against an
independent numpy restatement (tests/pyref.py) + libstdc++ sort model.

PARITY UNPINNED by the reference (no golden vectors exist upstream; the
reference cannot be compiled here). These tests pin the oracle against its own
committed fixtures and against a second, independently written restatement.
"""
import math
import os

import numpy as np
import pytest

import pyoracle as O
import pyref
from introsort_ref import sort_order_greater
from roborts_csm.params import CorrelationScanMatchParam


def _param(a):
    return CorrelationScanMatchParam(float(a[0]), float(a[1]), float(a[2]), float(a[3]), float(a[4]),
                                     int(a[5]), int(a[6]), bool(a[7]), int(a[8]))


@pytest.fixture(scope="module")
def f1(golden_dir):
    return np.load(os.path.join(golden_dir, "f1_config1.npz"))


@pytest.fixture(scope="module")
def f3(golden_dir):
    return np.load(os.path.join(golden_dir, "f3_ties.npz"))


def test_f1_oracle_reproduces_fixture(f1):
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    p = _param(f1["param"])
    c = O.world_to_map(m, f1["init_pose"])
    assert np.array_equal(c, f1["center"])
    sc = O.score_window(m, f1["points"], p, c, f1["scores"].size)
    assert np.array_equal(sc, f1["scores"])
    assert np.array_equal(O.sorted_order(m, f1["points"], p, c, sc.size), f1["order"])
    r, pose, cov, am, n = O.scan_match(m, f1["points"], p, f1["init_pose"], np.eye(3))
    assert r == f1["response"] and am == f1["argmax"] and n == sc.size
    assert np.array_equal(pose, f1["pose"]) and np.array_equal(cov, f1["cov"])


def test_f1_independent_restatement(f1):
    """numpy restatement == C++ oracle, bit for bit (scores and sort order)."""
    g = f1["grid"]
    p = _param(f1["param"])
    mres = 1 / (1.0 / float(f1["resolution"]))
    sc, *_ = pyref.window_scores(g, f1["points"], p, f1["center"], mres)
    assert np.array_equal(sc, f1["scores"])
    assert np.array_equal(pyref.sorted_order(sc), f1["order"])


def test_f1_window_shape(f1):
    # BASELINE config 1: 16 theta x 21^2 = 7056 candidates, B = 121
    p = _param(f1["param"])
    assert pyref.dims(p) == (16, 21)
    n = f1["points"].shape[0]
    assert n == 361 or n < 361
    step = n // (p.use_point_size - 1) if n >= 2 * p.use_point_size else 1
    assert len(range(0, n, step)) == (121 if n == 361 else len(range(0, n, step)))


def test_f3_ties_oracle_and_model(f3):
    m = O.Map(f3["grid"], float(f3["resolution"]), tuple(f3["offset"]))
    mres = 1 / (1.0 / float(f3["resolution"]))
    for tag in ("pen", "nopen", "fine"):
        p = _param(f3[f"{tag}_param"])
        c = O.world_to_map(m, f3["init_pose"])
        sc = O.score_window(m, f3["points"], p, c, f3[f"{tag}_scores"].size)
        assert np.array_equal(sc, f3[f"{tag}_scores"])
        order = O.sorted_order(m, f3["points"], p, c, sc.size)
        assert np.array_equal(order, f3[f"{tag}_order"])
        # independent: numpy scores + Python libstdc++ introsort model
        sc2, *_ = pyref.window_scores(f3["grid"], f3["points"], p, c, mres)
        assert np.array_equal(sc2, sc)
        assert np.array_equal(pyref.sorted_order(sc2), order)
        # the ties are real: the sort order is not the stable one
        if tag != "pen":
            stable = np.argsort(-sc, kind="stable")
            assert not np.array_equal(stable, order)


def test_f2_oracle_reproduces_fixture(golden_dir):
    f2 = np.load(os.path.join(golden_dir, "f2_config2_crop.npz"))
    m = O.Map(f2["grid"], float(f2["resolution"]), tuple(f2["offset"]))
    for tag in ("sim", "b1081", "pcfg"):
        levels = [_param(a) for a in f2[f"{tag}_levels"]]
        s, pose, cov = O.scan_matchers(m, f2["points"], levels, f2["init_pose"], np.eye(3))
        assert s == f2[f"{tag}_score"]
        assert np.array_equal(pose, f2[f"{tag}_pose"]) and np.array_equal(cov, f2[f"{tag}_cov"])
        for li in range(3):
            c = f2[f"{tag}_l{li}_center"]
            sc = O.score_window(m, f2["points"], levels[li], c, f2[f"{tag}_l{li}_scores"].size)
            assert np.array_equal(sc, f2[f"{tag}_l{li}_scores"])


def test_f4_bnb_fixture(golden_dir):
    f1 = np.load(os.path.join(golden_dir, "f1_config1.npz"))
    f4 = np.load(os.path.join(golden_dir, "f4_bnb.npz"))
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    r, pose, cov, _, n = O.scan_match(m, f1["points"], _param(f4["param"]), f1["init_pose"], np.eye(3))
    assert r == f4["response"] and n == f4["n_scored"]
    assert np.array_equal(pose, f4["pose"]) and np.array_equal(cov, f4["cov"])


def test_f5_large_window_fixture(golden_dir):
    f1 = np.load(os.path.join(golden_dir, "f1_config1.npz"))
    f5 = np.load(os.path.join(golden_dir, "f5_large_window.npz"))
    m = O.Map(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]))
    s, flat = O.best_window(m, f1["points"], _param(f5["param"]), f5["center"])
    assert s == f5["best_score"] and flat == f5["best_flat"]


def test_std_sort_model_matches_libstdcxx():
    rng = np.random.default_rng(3)
    for trial in range(60):
        n = int(rng.integers(1, 2500))
        k = rng.integers(0, int(rng.integers(1, 40)), size=n).astype(np.float64)
        assert np.array_equal(O.std_sort_order(k), np.array(sort_order_greater(k)))


def test_map_world_round_trip():
    m = O.Map(np.zeros((10, 10), np.float32), 0.05, (12.5, -3.25))
    for w in ([0.0, 0.0, 0.3], [1.234, -5.5, -2.0], [-12.5, 3.25, 0.0]):
        p = O.world_to_map(m, w)
        assert p[0] == 20.0 * w[0] + 20.0 * 12.5 and p[1] == 20.0 * w[1] + 20.0 * -3.25
        back = O.map_to_world(m, p)
        assert np.allclose(back, w, atol=1e-12, rtol=0)


def test_aos_cells_equal_packed(golden_dir):
    """The reference's 8-byte ProbabilityCell layout reads like a packed grid."""
    f1 = np.load(os.path.join(golden_dir, "f1_config1.npz"))
    g = f1["grid"]
    aos = np.zeros(g.shape, dtype=[("prob_value_", "<f4"), ("update_index_", "<i4")])
    aos["prob_value_"] = g
    aos["update_index_"] = -1
    m = O.Map(aos, float(f1["resolution"]), tuple(f1["offset"]))
    sc = O.score_window(m, f1["points"], _param(f1["param"]), f1["center"], f1["scores"].size)
    assert np.array_equal(sc, f1["scores"])
