"""Host logic of the v7 phase kernel (csm_phase.hip): the phase buckets the
library builds for a sub-cell window step (csm_api.cpp phase_table, through
the csm_phase_buckets hook). Checked in exact rational arithmetic, no GPU:
inside bucket q, candidate j reads column floor(t) + ox[q][j] for every
phase, at least the 2^-20 margin away from any column change
(correlate_scan_matcher.h:569-572 enumeration, :645-659 truncation); and
every phase comfortably away from all breakpoints lies in some bucket, so the
exact cell-by-cell path only takes beams near a breakpoint."""
import ctypes as C
import math
import random
from fractions import Fraction

import numpy as np
import pytest

from roborts_csm import _abi

_lib = _abi.load_library()
M = Fraction(1, 2 ** 20)


def buckets(f, ns, margin_log2=20):
    nq, cells = C.c_int32(), C.c_int32()
    lo = (C.c_double * 8)()
    hi = (C.c_double * 8)()
    ox = (C.c_int8 * 128)()
    st = _lib.csm_phase_buckets(f, ns, margin_log2, C.byref(nq), C.byref(cells), lo, hi, ox)
    if st != 0:
        return None
    oxa = np.frombuffer(ox, dtype=np.int8).reshape(8, 16)
    return nq.value, cells.value, list(lo), list(hi), oxa


def dist_to_int(x):
    return min(x - math.floor(x), math.ceil(x) - x)


# window steps of the shipped parameter sets on 5 cm and 2.5 cm maps, and others
STEPS = [(0.02 / 0.05, 11), (0.01 / 0.05, 3), (0.02 / 0.025, 11), (0.01 / 0.025, 3), (0.3, 4), (0.7, 3),
         (1 / 3, 13), (0.25, 16), (0.125, 5), (0.9, 2), (0.05, 1)]


@pytest.mark.parametrize("f,ns", STEPS)
def test_bucket_offsets_exact(f, ns):
    b = buckets(f, ns)
    assert b is not None
    nq, cells, lo, hi, ox = b
    F = Fraction(f)  # the exact double
    assert 1 <= nq <= 8
    assert cells == int(ox[:nq, :ns].max()) + 1 and int(ox[:nq, :ns].min()) >= 0
    for q in range(nq):
        l, h = Fraction(lo[q]), Fraction(hi[q])
        assert M <= l < h <= 1 - M
        if q:
            assert Fraction(hi[q - 1]) < l  # disjoint, ascending
        for j in range(ns):
            a, z = l + j * F, h + j * F
            assert math.floor(a) == math.floor(z) == int(ox[q, j]), (q, j)
            # no column change inside, and both ends at least a margin from one
            assert dist_to_int(a) >= M and dist_to_int(z) >= M, (q, j)


@pytest.mark.parametrize("f,ns", STEPS)
def test_buckets_cover_safe_phases(f, ns):
    nq, cells, lo, hi, ox = buckets(f, ns)
    F = Fraction(f)
    rng = random.Random(7)
    for _ in range(4000):
        p = Fraction(rng.random())
        if min(dist_to_int(p + j * F) for j in range(ns)) < Fraction(1, 2 ** 17):
            continue  # near a breakpoint: the exact path's
        inside = [q for q in range(nq) if Fraction(lo[q]) <= p <= Fraction(hi[q])]
        assert len(inside) == 1, p


def test_fine_level_shape():
    """The sim-YAML fine window on a 5 cm map is the instantiated kernel shape:
    f = 0.02 / 0.05 = 0.39999999999999997 (not 0.4: breakpoints 0 and 2e-16
    both appear and merge), 5 buckets, 5 x 5 boxes."""
    nq, cells, lo, hi, ox = buckets(0.02 / 0.05, 11)
    assert (nq, cells) == (5, 5)
    # offsets of bucket q: floor((q + 0.5) / 5 + 0.4 j)
    for q in range(5):
        assert list(ox[q, :11]) == [math.floor((q + 0.5) / 5 + 0.4 * j) for j in range(11)]


def test_unsupported_steps():
    assert buckets(1.0, 13) is None  # whole-cell steps: the box kernel's
    assert buckets(2.0, 11) is None
    assert buckets(0.4, 17) is None  # more positions than the table holds
    assert buckets(0.3, 9) is None  # ten buckets: more than the table holds
