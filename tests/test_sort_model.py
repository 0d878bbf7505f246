"""CPU: the std::sort tie-order models against libstdc++ itself.

tests/introsort_ref.py restates libstdc++'s introsort; tests/wave_sort_model.py
restates the formulation the device finish kernel computes (rank-paired
partition + per-segment stable sort). Both must reproduce the permutation
std::sort(greater) gives (correlate_scan_matcher.h:607) — ties included."""
import numpy as np
import pytest

import pyoracle as O
import wave_sort_model as W
from introsort_ref import sort_order_greater


def _cases(seed, n_cases):
    rng = np.random.default_rng(seed)
    for t in range(n_cases):
        n = int(rng.integers(1, 2500))
        k = rng.integers(0, int(rng.integers(1, 60)), size=n).astype(float)
        if t % 3 == 0:
            k = rng.random(n)
        if t % 5 == 0:
            k = np.sort(k)
        if t % 7 == 0:
            k = k[::-1].copy()
        yield k


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_device_formulation_matches_libstdcxx(seed):
    for k in _cases(seed, 60):
        assert np.array_equal(O.std_sort_order(k), np.array(W.device_sort_order(k)))


def test_all_equal_and_two_values():
    for n in (17, 64, 65, 1000, 5070):
        k = np.zeros(n)
        assert np.array_equal(O.std_sort_order(k), np.array(W.device_sort_order(k)))
        k = (np.arange(n) % 2).astype(float)
        assert np.array_equal(O.std_sort_order(k), np.array(sort_order_greater(k)))
        assert np.array_equal(O.std_sort_order(k), np.array(W.device_sort_order(k)))
