"""ORACLE — test infrastructure, not product code.

Only tests/ may import this module, and only as the checker.

Which candidates CPU torch.topk returns when scores tie. The reference's Recall@k takes
``torch.topk(user_item_scores_sampled, k, dim=1)`` (reference utils/train_test.py:197) and counts
the positives among the returned indices (:200-204). Candidate rows repeat (an item that is the
positive of one validation edge and a sampled negative of another has the same row, hence the same
score), so several candidates can share the k-th score, and which of them are returned decides hits.
On a CPU, torch 2.10's topk is ATen's ``topk_impl_loop`` (aten/src/ATen/native/TopKImpl.h): the row
as (value, index) pairs, then

    use_partial_sort = k * 64 <= n
    std::partial_sort(q, q + k, q + n, comp)          if use_partial_sort
    std::nth_element(q, q + k - 1, q + n, comp)       otherwise (then std::sort of the first k - 1)
    comp(x, y) = (isnan(x) && !isnan(y)) || x > y     (largest = True)

with libstdc++'s algorithms (torch's wheel: GCC 11.2, ``torch.__config__.show()``). The returned
set is the first k slots. This module restates those libstdc++ routines step for step
(bits/stl_heap.h: __adjust_heap, __push_heap, __make_heap, __pop_heap; bits/stl_algo.h:
__heap_select, __move_median_to_first, __unguarded_partition, __insertion_sort,
__unguarded_linear_insert, __introselect). Pinned against torch.topk itself on tie-heavy rows in
tests/test_recall_stl.py (CPU) — torch is present here, so the pin is the real function, not a
fixture. csrc/lgcn_recall.hip's lgcn_select_topk_stl runs the same steps on the GPU.
"""
from __future__ import annotations

import math

import numpy as np


def _comp(x, y) -> bool:
    a, b = x[0], y[0]
    return (math.isnan(a) and not math.isnan(b)) or a > b


def _adjust_heap(a, first, hole, length, value):
    top = hole
    second = hole
    while second < (length - 1) // 2:
        second = 2 * (second + 1)
        if _comp(a[first + second], a[first + second - 1]):
            second -= 1
        a[first + hole] = a[first + second]
        hole = second
    if (length & 1) == 0 and second == (length - 2) // 2:
        second = 2 * (second + 1)
        a[first + hole] = a[first + second - 1]
        hole = second - 1
    parent = (hole - 1) // 2
    while hole > top and _comp(a[first + parent], value):
        a[first + hole] = a[first + parent]
        hole = parent
        parent = (hole - 1) // 2
    a[first + hole] = value


def _make_heap(a, first, last):
    n = last - first
    if n < 2:
        return
    parent = (n - 2) // 2
    while True:
        _adjust_heap(a, first, parent, n, a[first + parent])
        if parent == 0:
            return
        parent -= 1


def _heap_select(a, first, middle, last):
    _make_heap(a, first, middle)
    for i in range(middle, last):
        if _comp(a[i], a[first]):
            v = a[i]
            a[i] = a[first]
            _adjust_heap(a, first, 0, middle - first, v)


def _move_median_to_first(a, r, x, y, z):
    if _comp(a[x], a[y]):
        if _comp(a[y], a[z]):
            a[r], a[y] = a[y], a[r]
        elif _comp(a[x], a[z]):
            a[r], a[z] = a[z], a[r]
        else:
            a[r], a[x] = a[x], a[r]
    elif _comp(a[x], a[z]):
        a[r], a[x] = a[x], a[r]
    elif _comp(a[y], a[z]):
        a[r], a[z] = a[z], a[r]
    else:
        a[r], a[y] = a[y], a[r]


def _unguarded_partition(a, first, last, pivot):
    while True:
        while _comp(a[first], a[pivot]):
            first += 1
        last -= 1
        while _comp(a[pivot], a[last]):
            last -= 1
        if not first < last:
            return first
        a[first], a[last] = a[last], a[first]
        first += 1


def _insertion_sort(a, first, last):
    if first == last:
        return
    for i in range(first + 1, last):
        v = a[i]
        if _comp(v, a[first]):
            a[first + 1:i + 1] = a[first:i]  # std::move_backward
            a[first] = v
        else:
            j, nxt = i, i - 1
            while _comp(v, a[nxt]):
                a[j] = a[nxt]
                j = nxt
                nxt -= 1
            a[j] = v


def _nth_element(a, first, nth, last):
    if first == last or nth == last:
        return
    depth = 2 * ((last - first).bit_length() - 1)  # 2 * std::__lg(n)
    while last - first > 3:
        if depth == 0:
            _heap_select(a, first, nth + 1, last)
            a[first], a[nth] = a[nth], a[first]
            return
        depth -= 1
        mid = first + (last - first) // 2
        _move_median_to_first(a, first, first + 1, mid, last - 1)
        cut = _unguarded_partition(a, first + 1, last, first)
        if cut <= nth:
            first = cut
        else:
            last = cut
    _insertion_sort(a, first, last)


def topk_indices(row, k: int) -> np.ndarray:
    """The index SET CPU torch.topk(row, k) returns (sorted ascending), row a 1-D float array."""
    a = [(float(v), i) for i, v in enumerate(np.asarray(row, dtype=np.float32))]
    n = len(a)
    if not 0 < k <= n:
        raise RuntimeError("selected index k out of range")
    if k * 64 <= n:
        _heap_select(a, 0, k, n)  # std::partial_sort = __heap_select + __sort_heap (same set)
    else:
        _nth_element(a, 0, k - 1, n)
    return np.sort(np.fromiter((i for _, i in a[:k]), dtype=np.int64, count=k))


def topk_hits(scores: np.ndarray, k: int, P: int) -> np.ndarray:
    """Per row of scores [Q, M] (float32): positives (index < P) among CPU torch.topk's k."""
    return np.array([int((topk_indices(r, k) < P).sum()) for r in np.asarray(scores)], dtype=np.int64)
