"""CPU oracle for the config-5 caller's per-pixel channel statistics (ChannelPool).

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (``admmtor``) may import, call or
execute this file; only ``tests/`` use it, as the checker of the HIP kernel of
``include/admm_chanstat.h``.

Restates ``ChannelPool.forward`` (``/root/reference/src/admmtor/elayers/attentions.py:44-47``):

    cat(std(x, 1), median(x, 1).values, mode(x, 1).values)

whose arithmetic lives in PyTorch's CPU kernels (the reference pins torch 2.4.1):

* ``std``: unbiased (correction 1), rounded to the input dtype;
* ``median``: the lower median; its index (where the gradient goes) is the element at
  position (C-1)//2 of a STABLE ascending sort -- ties broken by channel index;
* ``mode``: PyTorch's CPU mode kernel copies the (value, channel) pairs, runs libstdc++
  ``std::sort`` on them with the comparator ``a.first < b.first`` and scans the sorted pairs
  for the first longest run of equal values, returning the value and channel of the LAST pair
  of that run.  ``std::sort`` (introsort) is not stable for more than 16 elements, so the
  returned channel is whatever the introsort leaves last in the run: :func:`std_sort` restates
  libstdc++'s algorithm (bits/stl_algo.h ``__introsort_loop``, ``__unguarded_partition_pivot``,
  ``__move_median_to_first``, ``__unguarded_partition``, ``__final_insertion_sort``;
  bits/stl_heap.h ``__adjust_heap``, ``__push_heap``, ``make_heap``/``sort_heap`` for the
  depth-limit fallback) step for step.

Pinning: ``tests/test_chanpool_oracle.py`` checks this restatement against torch's own CPU
``median``/``mode`` values and indices on heavy-tie inputs (C = 1 ... 200) and against the
committed fixture ``tests/golden/g9_chanpool.npz`` (written by ``tests/golden/make_golden_chanpool.py``
from torch's CPU kernels); the heapsort fallback (reached only through the depth budget) is
checked against ``std::make_heap`` + ``std::sort_heap`` compiled here with g++.
NaN inputs: the mode is unpinned (``<`` is not a strict weak order with NaN); the median of a
column holding NaN is its first NaN (torch.median's rule), which the GPU tests check against
torch's CPU kernels directly.
"""
from __future__ import annotations

import numpy as np

THRESHOLD = 16  # libstdc++ _S_threshold


def _adjust_heap(a, f, hole, n, v):
    top = hole
    sc = hole
    while sc < (n - 1) // 2:
        sc = 2 * (sc + 1)
        if a[f + sc][0] < a[f + sc - 1][0]:
            sc -= 1
        a[f + hole] = a[f + sc]
        hole = sc
    if (n & 1) == 0 and sc == (n - 2) // 2:
        sc = 2 * (sc + 1)
        a[f + hole] = a[f + sc - 1]
        hole = sc - 1
    parent = (hole - 1) // 2 if hole > 0 else 0  # C++ truncation: (0 - 1) / 2 == 0
    while hole > top and a[f + parent][0] < v[0]:
        a[f + hole] = a[f + parent]
        hole = parent
        parent = (hole - 1) // 2 if hole > 0 else 0
    a[f + hole] = v


def heap_sort(a, f, l):
    """std::__partial_sort(f, l, l) == std::make_heap(f, l) then std::sort_heap(f, l)."""
    n = l - f
    if n >= 2:
        parent = (n - 2) // 2
        while True:
            _adjust_heap(a, f, parent, n, a[f + parent])
            if parent == 0:
                break
            parent -= 1
    last = l
    while last - f > 1:
        last -= 1
        v = a[last]
        a[last] = a[f]
        _adjust_heap(a, f, 0, last - f, v)


def _partition_pivot(a, f, l):
    mid = f + (l - f) // 2
    va, vb, vc = a[f + 1][0], a[mid][0], a[l - 1][0]
    if va < vb:
        sel = mid if vb < vc else (l - 1 if va < vc else f + 1)
    else:
        sel = f + 1 if va < vc else (l - 1 if vb < vc else mid)
    a[f], a[sel] = a[sel], a[f]
    pv = a[f][0]
    i, j = f + 1, l
    while True:
        while a[i][0] < pv:
            i += 1
        j -= 1
        while pv < a[j][0]:
            j -= 1
        if not i < j:
            return i
        a[i], a[j] = a[j], a[i]
        i += 1


def _introsort_loop(a, f, l, depth, stats):
    while l - f > THRESHOLD:
        if depth == 0:
            stats["heapsort"] += 1
            heap_sort(a, f, l)
            return
        depth -= 1
        cut = _partition_pivot(a, f, l)
        _introsort_loop(a, cut, l, depth, stats)
        l = cut


def std_sort(pairs, depth_limit=None, stats=None):
    """libstdc++ std::sort of a list of (value, channel) pairs by value, in place; returns it.
    ``depth_limit`` overrides 2*floor(log2 n) (the kernel's test hook does the same)."""
    n = len(pairs)
    stats = stats if stats is not None else {"heapsort": 0}
    if n > 1:
        depth = 2 * (n.bit_length() - 1) if depth_limit is None else depth_limit
        _introsort_loop(pairs, 0, n, depth, stats)
        for i in range(1, n):  # __final_insertion_sort
            v = pairs[i]
            j = i
            while j > 0 and v[0] < pairs[j - 1][0]:
                pairs[j] = pairs[j - 1]
                j -= 1
            pairs[j] = v
    return pairs


def mode_of(column, depth_limit=None):
    """torch.mode on the CPU for one 1-D column -> (value, channel)."""
    pairs = std_sort([(float(v), c) for c, v in enumerate(column)], depth_limit)
    best, run, out = 0, 0, pairs[0]
    for i in range(len(pairs)):
        run += 1
        if i == len(pairs) - 1 or pairs[i][0] != pairs[i + 1][0]:
            if run > best:
                best, out = run, pairs[i]
            run = 0
    return out


def median_of(column):
    """torch.median on the CPU for one 1-D column -> (value, channel): stable rank (C-1)//2."""
    order = sorted(range(len(column)), key=lambda c: (float(column[c]), c))
    c = order[(len(column) - 1) // 2]
    return float(column[c]), c


def channel_pool(x: np.ndarray, depth_limit=None):
    """x (B, C, H, W) float array (the values of the input dtype, as float64) ->
    (std (B,H,W) float64 unrounded, median value/index, mode value/index (B,H,W))."""
    B, C, H, W = x.shape
    cols = np.moveaxis(x.astype(np.float64), 1, -1).reshape(-1, C)
    std = cols.std(axis=1, ddof=1) if C > 1 else np.full(cols.shape[0], np.nan)
    med = np.array([median_of(col) for col in cols])
    mod = np.array([mode_of(col, depth_limit) for col in cols])
    shp = (B, H, W)
    return (std.reshape(shp), med[:, 0].reshape(shp), med[:, 1].astype(np.int64).reshape(shp),
            mod[:, 0].reshape(shp), mod[:, 1].astype(np.int64).reshape(shp))


def channel_pool_backward(x: np.ndarray, std_out: np.ndarray, mi: np.ndarray, oi: np.ndarray, g: np.ndarray):
    """fp64 gradient of the three statistics (the reference's std_backward and
    value_selecting_reduction_backward; a zero std contributes no gradient): x (B,C,H,W), std_out (B,H,W) the forward's std,
    mi/oi (B,H,W) channels, g (B,3,H,W) -> (B,C,H,W)."""
    B, C, H, W = x.shape
    x = x.astype(np.float64)
    mean = x.mean(axis=1, keepdims=True)
    sd = std_out[:, None]
    # std_backward masks the division where the std is 0 (grad / (2 std)).masked_fill_(std == 0, 0)
    scale = np.divide(g[:, 0:1], (C - 1) * sd, out=np.zeros_like(sd, dtype=np.float64), where=sd != 0)
    gx = scale * (x - mean)
    ch = np.arange(C)[None, :, None, None]
    gx = gx + (ch == mi[:, None]) * g[:, 1:2] + (ch == oi[:, None]) * g[:, 2:3]
    return gx
