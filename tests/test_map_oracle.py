"""CPU: the map-building oracle (oracle/map_oracle.cpp, SURVEY.md 8f rows f1,
f4) against the independent Python restatement (tests/map_pyref.py) on every
map scenario, plus the kernels' closed-form Bresenham against the reference's
loop. Parity of the oracle with the reference is unpinned (no reference map
tests; unbuildable here): these two restatements pin each other."""
import numpy as np
import pytest

import map_scenarios as S
from map_engines import OracleEngine, PyrefEngine, same_state
from map_pyref import bresenham, bresenham_closed_form


@pytest.fixture(scope="module")
def scans():
    return S.make_scans(4)


@pytest.mark.parametrize("name", sorted(S.scenarios()))
def test_oracle_matches_pyref(name, scans):
    sc = S.scenarios()[name]
    a, pa = S.run(OracleEngine, sc, *scans)
    b, pb = S.run(PyrefEngine, sc, *scans)
    same_state(a, b)
    assert pa == pb


def test_growth_and_quirks_exercised(scans):
    sc = S.scenarios()["prob_blur_grow"]
    a, _ = S.run(OracleEngine, sc, *scans)
    st = a.state()
    assert st["size_x"] > sc["size"][0] and st["size_y"] > sc["size"][1]  # grew both ways
    # a growth attempt leaves the scan undrawn but advances cur_update_index
    assert st["cur_update_index"] > 3 * (st["map_update_index"] + 1)
    p = a.arrays()[0]
    # never-reset map: fresh cells are kDefaultCellProb, element 0 the map default
    assert p.ravel()[0] == np.float32(0.3) and np.any(p == np.float32(0.5))


def test_full_update_with_blur_oracle_only(scans):
    """The order-dependent combination the reference never uses: oracle and
    pyref agree; the device rejects it (tests/test_gpu_gridmap.py)."""
    sc = dict(S.scenarios()["prob_lines_grow"])
    sc["ops"] = [("update", k, True) for k in range(2)]
    a, _ = S.run(OracleEngine, sc, *scans)
    b, _ = S.run(PyrefEngine, sc, *scans)
    same_state(a, b)


def test_bresenham_closed_form():
    import pyoracle as O
    rng = np.random.default_rng(3)
    cases = [(0, 0, 0, 0), (0, 0, 5, 2), (5, 2, 0, 0), (0, 0, 2, 5), (3, 3, -4, 9), (-7, 1, 6, -3)]
    cases += [tuple(int(v) for v in rng.integers(-300, 300, 4)) for _ in range(400)]
    for c in cases:
        ref = bresenham(*c)
        assert bresenham_closed_form(*c) == ref, c
        assert [tuple(p) for p in O.bresenham(*c)] == ref, c
