"""Python model of the device finish's parallel std::sort emulation
(roborts-edu-slam_amd/csrc/csm_finish.hip): explicit segment stack, median-of-3
by one lane, the unguarded partition computed from rank-paired stop lists,
heap sort at depth 0, then a stable insertion sort of every segment.
Checked against libstdc++ (oracle) and tests/introsort_ref.py."""
from __future__ import annotations

import introsort_ref as R


def device_sort_order(keys) -> list:
    a = [(float(k), i) for i, k in enumerate(keys)]
    n = len(a)
    if n == 0:
        return []
    gt = lambda x, y: x[0] > y[0]
    starts = set()
    stack = [(0, n, 2 * (n.bit_length() - 1))]
    while stack:
        first, last, depth = stack.pop()
        starts.add(first)
        ln = last - first
        if ln <= 16:
            continue
        if depth == 0:
            R._heap_sort(a, first, last, gt)
            continue
        R._move_median_to_first(a, first, first + 1, first + ln // 2, last - 1, gt)
        P = a[first]
        lpos = [p for p in range(first + 1, last) if not gt(a[p], P)]
        rpos = [p for p in range(last - 1, first, -1) if not gt(P, a[p])]
        npairs = 0
        while npairs < min(len(lpos), len(rpos)) and lpos[npairs] < rpos[npairs]:
            npairs += 1
        cut = 1 << 60
        if npairs < len(lpos):
            cut = lpos[npairs]
        if npairs >= 1:
            cut = min(cut, rpos[npairs - 1])
        for k in range(npairs):
            i, j = lpos[k], rpos[k]
            a[i], a[j] = a[j], a[i]
        stack.append((cut, last, depth - 1))
        stack.append((first, cut, depth - 1))
    st = sorted(starts) + [n]
    for s, e in zip(st[:-1], st[1:]):
        seg = a[s:e]
        # stable insertion sort (== sorted by key desc, stable)
        for i in range(1, len(seg)):
            v = seg[i]
            j = i
            while j > 0 and gt(v, seg[j - 1]):
                seg[j] = seg[j - 1]
                j -= 1
            seg[j] = v
        a[s:e] = seg
    return [i for _, i in a]
