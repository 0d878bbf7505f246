"""Pure-Python model of libstdc++'s std::sort (introsort), used to pin the
candidate tie order the reference inherits from std::sort(greater)
(correlate_scan_matcher.h:607) independently of the C++ oracle.

Published algorithm (GCC libstdc++ bits/stl_algo.h, unchanged since GCC 4.x):
introsort loop with threshold 16 and depth limit 2*floor(log2 n); pivot =
median of (first+1, mid, last-1) moved to first; unguarded Hoare partition;
heap sort when the depth limit is hit; final insertion sort (guarded on the
first 16 elements, unguarded after). `comp(a, b)` is "a goes before b".
"""
from __future__ import annotations

_THRESHOLD = 16


def _lg(n: int) -> int:
    return n.bit_length() - 1


def std_sort(a: list, comp) -> None:
    n = len(a)
    if n == 0:
        return
    _introsort_loop(a, 0, n, 2 * _lg(n), comp)
    _final_insertion_sort(a, 0, n, comp)


def _introsort_loop(a, first, last, depth, comp):
    while last - first > _THRESHOLD:
        if depth == 0:
            _heap_sort(a, first, last, comp)
            return
        depth -= 1
        cut = _partition_pivot(a, first, last, comp)
        _introsort_loop(a, cut, last, depth, comp)
        last = cut


def _move_median_to_first(a, result, x, y, z, comp):
    if comp(a[x], a[y]):
        if comp(a[y], a[z]):
            a[result], a[y] = a[y], a[result]
        elif comp(a[x], a[z]):
            a[result], a[z] = a[z], a[result]
        else:
            a[result], a[x] = a[x], a[result]
    elif comp(a[x], a[z]):
        a[result], a[x] = a[x], a[result]
    elif comp(a[y], a[z]):
        a[result], a[z] = a[z], a[result]
    else:
        a[result], a[y] = a[y], a[result]


def _partition_pivot(a, first, last, comp):
    mid = first + (last - first) // 2
    _move_median_to_first(a, first, first + 1, mid, last - 1, comp)
    return _unguarded_partition(a, first + 1, last, first, comp)


def _unguarded_partition(a, first, last, pivot, comp):
    while True:
        while comp(a[first], a[pivot]):
            first += 1
        last -= 1
        while comp(a[pivot], a[last]):
            last -= 1
        if not first < last:
            return first
        a[first], a[last] = a[last], a[first]
        first += 1


def _unguarded_linear_insert(a, last, comp):
    val = a[last]
    nxt = last - 1
    while comp(val, a[nxt]):
        a[last] = a[nxt]
        last = nxt
        nxt -= 1
    a[last] = val


def _insertion_sort(a, first, last, comp):
    if first == last:
        return
    for i in range(first + 1, last):
        if comp(a[i], a[first]):
            val = a[i]
            a[first + 1:i + 1] = a[first:i]
            a[first] = val
        else:
            _unguarded_linear_insert(a, i, comp)


def _final_insertion_sort(a, first, last, comp):
    if last - first > _THRESHOLD:
        _insertion_sort(a, first, first + _THRESHOLD, comp)
        for i in range(first + _THRESHOLD, last):
            _unguarded_linear_insert(a, i, comp)
    else:
        _insertion_sort(a, first, last, comp)


# -- heap sort (__partial_sort(first, last, last) = make_heap + sort_heap) ----

def _push_heap(a, base, hole, top, val, comp):
    parent = (hole - 1) // 2
    while hole > top and comp(a[base + parent], val):
        a[base + hole] = a[base + parent]
        hole = parent
        parent = (hole - 1) // 2
    a[base + hole] = val


def _adjust_heap(a, base, hole, length, val, comp):
    top = hole
    second = hole
    while second < (length - 1) // 2:
        second = 2 * (second + 1)
        if comp(a[base + second], a[base + second - 1]):
            second -= 1
        a[base + hole] = a[base + second]
        hole = second
    if (length & 1) == 0 and second == (length - 2) // 2:
        second = 2 * (second + 1)
        a[base + hole] = a[base + second - 1]
        hole = second - 1
    _push_heap(a, base, hole, top, val, comp)


def _heap_sort(a, first, last, comp):
    length = last - first
    if length >= 2:
        parent = (length - 2) // 2
        while True:
            _adjust_heap(a, first, parent, length, a[first + parent], comp)
            if parent == 0:
                break
            parent -= 1
    while last - first > 1:
        last -= 1
        val = a[last]
        a[last] = a[first]
        _adjust_heap(a, first, 0, last - first, val, comp)


def sort_order_greater(keys) -> list:
    """Indices in the order std::sort(greater-by-key) leaves them."""
    a = [(float(k), i) for i, k in enumerate(keys)]
    std_sort(a, lambda x, y: x[0] > y[0])
    return [i for _, i in a]
