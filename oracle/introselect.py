"""Restatement of ``torch.topk(x, k, largest=True, sorted=False)`` on CPU — the
resample step of the reference (dgc/compression.py:134-137) — down to the ORDER of
the returned indices, which is the order of the transmitted (values, indices).

TEST INFRASTRUCTURE ONLY (imported by ``oracle/dgc_oracle.py`` and ``tests/``);
the product path never imports it.

Third-party algorithm. The reference calls PyTorch (torch>=1.5, requirements.txt:1;
pinned here: torch 2.10.0 CPU). Its CPU topk (aten/src/ATen/native/cpu/SortingKernel.cpp,
``topk_impl_loop``) fills ``queue[j] = (x[j], j)`` and runs, with the comparator
``comp(a, b) = (isnan(a) and not isnan(b)) or a > b`` on the values only:

* ``k * 64 <= n``: ``std::partial_sort(queue, queue + k, queue + n, comp)``;
* otherwise ``std::nth_element(queue, queue + k - 1, queue + n, comp)``;

and returns ``queue[0:k]``'s indices in that order. Both are libstdc++'s algorithms
(introselect with median-of-3 and Hoare partitioning; heap select + sort_heap), which
this file restates. tests/test_introselect.py checks it against torch.topk itself on
thousands of tie-heavy inputs, and tests/test_oracle_golden.py against the reference's
golden resample steps, in order.

The nth_element partition is written in the same data-parallel form the GPU kernel
(K5: ``adam-compression_amd/csrc/introselect.hpp``, launched from ``csrc/select.hip``'s
``k_nth_select`` / ``k_nth_global``) uses, so this file is also that kernel's
specification; ``partial_sort`` below is what K5b (``heap_select_wg`` in
``csrc/select.hip``) replays. One
``__unguarded_partition(first + 1, last, pivot = first)`` is, with P the pivot key:

    L_1 < L_2 < ...  positions in [first+1, last) with key <= P  (left scan stops)
    R_1 > R_2 > ...  positions in [first,   last) with key >= P  (right scan stops;
                     the pivot slot itself stops it)
    s   = #{t : L_t < R_t}          (the swaps performed: L_t <-> R_t, t <= s)
    cut = min(L_{s+1}, R_s)         (R_0 = last; L_{s+1} = +inf if it does not exist)

because every swap puts a left-stopper at R_t and a right-stopper at L_t, which end
the next scans at the latest there. Keys are |x| bit patterns (non-negative, so
unsigned order is float order); NaN keys are made equal, as comp makes them.
"""
import numpy as np

__all__ = ["keys_of", "nth_element", "partial_sort", "topk_order"]


def keys_of(values):
    """uint32 sort keys: |x| bits with every NaN mapped to one key above +inf."""
    a = np.abs(np.asarray(values, dtype=np.float32)).view(np.uint32).copy()
    a[a > 0x7F800000] = 0x7FC00000
    return a


def _lg(n):
    return int(n).bit_length() - 1


# ------------------------------------------------------------------ nth_element
def _median_to_first(key, pos, f, a, b, c):
    """std::__move_median_to_first(result=f, a, b, c) with comp = key greater."""
    ka, kb, kc = key[a], key[b], key[c]
    if ka > kb:
        if kb > kc:
            m = b
        elif ka > kc:
            m = c
        else:
            m = a
    elif ka > kc:
        m = a
    elif kb > kc:
        m = c
    else:
        m = b
    key[f], key[m] = key[m], key[f]
    pos[f], pos[m] = pos[m], pos[f]


def _partition(key, pos, f, l):
    """std::__unguarded_partition(f + 1, l, pivot = f) in parallel form; returns the cut."""
    P = key[f]
    lb = np.flatnonzero(key[f + 1:l] <= P) + (f + 1)          # L_1 < L_2 < ...
    rb = (np.flatnonzero(key[f:l] >= P) + f)[::-1]            # R_1 > R_2 > ...
    m = min(lb.size, rb.size)
    crossed = lb[:m] >= rb[:m]
    s = int(np.argmax(crossed)) if crossed.any() else m
    L_next = int(lb[s]) if s < lb.size else np.iinfo(np.int64).max
    R_last = int(rb[s - 1]) if s > 0 else l
    if s:
        li, ri = lb[:s], rb[:s]
        key[li], key[ri] = key[ri].copy(), key[li].copy()
        pos[li], pos[ri] = pos[ri].copy(), pos[li].copy()
    return min(L_next, R_last)


def _insertion_sort(key, pos, f, l):
    """std::__insertion_sort with std::__unguarded_linear_insert (ranges of <= 3)."""
    for i in range(f + 1, l):
        kv, pv = key[i], pos[i]
        if kv > key[f]:
            key[f + 1:i + 1] = key[f:i].copy()
            pos[f + 1:i + 1] = pos[f:i].copy()
            key[f], pos[f] = kv, pv
        else:
            j = i - 1
            while kv > key[j]:
                key[j + 1], pos[j + 1] = key[j], pos[j]
                j -= 1
            key[j + 1], pos[j + 1] = kv, pv


# ------------------------------------------------------------------ heaps
def _adjust_heap(key, pos, f, hole, n, kv, pv):
    """std::__adjust_heap + std::__push_heap on [f, f + n) with comp = key greater."""
    top = hole
    child = hole
    while child < (n - 1) // 2:
        child = 2 * (child + 1)
        if key[f + child] > key[f + child - 1]:
            child -= 1
        key[f + hole], pos[f + hole] = key[f + child], pos[f + child]
        hole = child
    if (n & 1) == 0 and child == (n - 2) // 2:
        child = 2 * (child + 1)
        key[f + hole], pos[f + hole] = key[f + child - 1], pos[f + child - 1]
        hole = child - 1
    parent = (hole - 1) // 2
    while hole > top and key[f + parent] > kv:
        key[f + hole], pos[f + hole] = key[f + parent], pos[f + parent]
        hole = parent
        parent = (hole - 1) // 2
    key[f + hole], pos[f + hole] = kv, pv


def _make_heap(key, pos, f, l):
    n = l - f
    if n < 2:
        return
    parent = (n - 2) // 2
    while True:
        _adjust_heap(key, pos, f, parent, n, key[f + parent], pos[f + parent])
        if parent == 0:
            return
        parent -= 1


def _pop_heap(key, pos, f, l, r):
    kv, pv = key[r], pos[r]
    key[r], pos[r] = key[f], pos[f]
    _adjust_heap(key, pos, f, 0, l - f, kv, pv)


def _heap_select(key, pos, f, mid, l):
    _make_heap(key, pos, f, mid)
    for i in range(mid, l):
        if key[i] > key[f]:
            _pop_heap(key, pos, f, mid, i)


def _sort_heap(key, pos, f, l):
    while l - f > 1:
        l -= 1
        _pop_heap(key, pos, f, l, l)


# ------------------------------------------------------------------ entry points
def nth_element(key, pos, nth):
    """std::nth_element(queue, queue + nth, queue + n, comp), in place."""
    f, l = 0, key.size
    if f == l or nth == l:
        return
    depth = 2 * _lg(l - f)
    while l - f > 3:
        if depth == 0:
            _heap_select(key, pos, f, nth + 1, l)
            key[f], key[nth] = key[nth], key[f]
            pos[f], pos[nth] = pos[nth], pos[f]
            return
        depth -= 1
        _median_to_first(key, pos, f, f + 1, f + (l - f) // 2, l - 1)
        cut = _partition(key, pos, f, l)
        if cut <= nth:
            f = cut
        else:
            l = cut
    _insertion_sort(key, pos, f, l)


def partial_sort(key, pos, k):
    """std::partial_sort(queue, queue + k, queue + n, comp), in place."""
    _heap_select(key, pos, 0, k, key.size)
    _sort_heap(key, pos, 0, k)


def topk_order(values, k):
    """``torch.topk(values, k, largest=True, sorted=False)[1]`` on CPU (int64)."""
    key = keys_of(values).astype(np.int64)
    n = key.size
    pos = np.arange(n, dtype=np.int64)
    if k <= 0:
        return pos[:0]
    if k * 64 <= n:
        partial_sort(key, pos, k)
    else:
        nth_element(key, pos, k - 1)
    return pos[:k].copy()
