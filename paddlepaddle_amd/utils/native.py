"""Access to the native C++ runtime module ``_C_runtime`` (built by tools/build_native.py).

It hosts the CPU-side runtime pieces the reference implements in C++: batch collation for the
DataLoader, the static-graph scheduler (topological order, liveness/last-use analysis, dependency
levels) used by ``static.Executor``, gradient-bucket planning for DataParallel/sharding, and a fast
tensor-file writer for checkpoints. Every entry point has a pure-Python fallback so the package
imports on machines where the module was not built, but ``build()`` always builds it.
"""
from __future__ import annotations

import importlib
import os
import sys

import numpy as np

_mod = None
_err = None


def module():
    global _mod, _err
    if _mod is not None or _err is not None:
        return _mod
    try:
        _mod = importlib.import_module("paddlepaddle_amd._C_runtime")
    except ImportError as e:
        _err = str(e)
        _mod = None
    return _mod


def available():
    return module() is not None


def stack_arrays(arrs):
    m = module()
    if m is not None and arrs and all(isinstance(a, np.ndarray) for a in arrs):
        a0 = arrs[0]
        if all(a.shape == a0.shape and a.dtype == a0.dtype for a in arrs) and a0.dtype.kind in "fiub":
            out = np.empty((len(arrs),) + a0.shape, a0.dtype)
            m.stack_into([np.ascontiguousarray(a) for a in arrs], out)
            return out
    return np.stack(arrs)


def plan_buckets(sizes_bytes, bucket_bytes):
    """Greedy reverse-order bucketing: returns list of lists of indices."""
    m = module()
    if m is not None:
        return m.plan_buckets(list(int(s) for s in sizes_bytes), int(bucket_bytes))
    buckets, cur, cur_b = [], [], 0
    for i in reversed(range(len(sizes_bytes))):
        cur.append(i)
        cur_b += sizes_bytes[i]
        if cur_b >= bucket_bytes:
            buckets.append(cur)
            cur, cur_b = [], 0
    if cur:
        buckets.append(cur)
    return buckets


def schedule(n_nodes, edges, outputs_keep, prio=None):
    """Topological schedule of a DAG. edges: list of (src, dst). Among ready nodes the lowest ``prio`` class
    goes first, then the smallest id. Returns (order, last_use) where last_use[v] is the position in
    ``order`` after which value v can be freed (-1 = keep)."""
    m = module()
    prio = list(prio) if prio is not None else []
    if m is not None:
        return m.schedule(int(n_nodes), [(int(a), int(b)) for a, b in edges], list(int(k) for k in outputs_keep),
                          [int(x) for x in prio])
    cls = (lambda v: prio[v]) if len(prio) == n_nodes else (lambda v: 0)
    indeg = [0] * n_nodes
    succ = [[] for _ in range(n_nodes)]
    for a, b in edges:
        succ[a].append(b)
        indeg[b] += 1
    import heapq
    ready = [(cls(i), i) for i in range(n_nodes) if indeg[i] == 0]
    heapq.heapify(ready)
    order = []
    while ready:
        _, v = heapq.heappop(ready)
        order.append(v)
        for w in succ[v]:
            indeg[w] -= 1
            if indeg[w] == 0:
                heapq.heappush(ready, (cls(w), w))
    if len(order) != n_nodes:
        raise ValueError("graph has a cycle")
    pos = {v: i for i, v in enumerate(order)}
    keep = set(outputs_keep)
    last = [-1] * n_nodes
    for v in range(n_nodes):
        if v in keep:
            continue
        last[v] = max([pos[w] for w in succ[v]], default=pos[v])
    return order, last
