"""paddle.geometric: message passing, segment reductions, graph sampling.
Reference: python/paddle/geometric/ (message_passing/send_recv.py: send_u_recv, send_ue_recv, send_uv;
math.py: segment_sum/mean/max/min; reindex.py; sampling/neighbors.py).
Reductions are device scatter-reduce (index_reduce / scatter_reduce) over the destination index."""
from __future__ import annotations

import numpy as np
import torch

from ..framework.tensor import Tensor, _wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else torch.as_tensor(x)


def _reduce(src, index, n, op):
    shape = (n,) + tuple(src.shape[1:])
    idx = index.long().view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    if op == "sum":
        return torch.zeros(shape, dtype=src.dtype, device=src.device).scatter_add_(0, idx, src)
    if op == "mean":
        s = torch.zeros(shape, dtype=src.dtype, device=src.device).scatter_add_(0, idx, src)
        c = torch.zeros(n, dtype=src.dtype, device=src.device).scatter_add_(0, index.long(),
                                                                             torch.ones_like(index, dtype=src.dtype))
        return s / c.clamp_min(1).view(-1, *([1] * (src.dim() - 1)))
    if op in ("max", "min"):
        fill = float("-inf") if op == "max" else float("inf")
        out = torch.full(shape, fill, dtype=src.dtype, device=src.device)
        out = out.scatter_reduce(0, idx, src, reduce="amax" if op == "max" else "amin", include_self=True)
        return torch.where(torch.isinf(out), torch.zeros_like(out), out)
    raise ValueError(op)


def segment_sum(data, segment_ids, name=None):
    d, s = _t(data), _t(segment_ids)
    n = int(s.max()) + 1 if s.numel() else 0
    return _wrap(_reduce(d, s, n, "sum"))


def segment_mean(data, segment_ids, name=None):
    d, s = _t(data), _t(segment_ids)
    n = int(s.max()) + 1 if s.numel() else 0
    return _wrap(_reduce(d, s, n, "mean"))


def segment_max(data, segment_ids, name=None):
    d, s = _t(data), _t(segment_ids)
    n = int(s.max()) + 1 if s.numel() else 0
    return _wrap(_reduce(d, s, n, "max"))


def segment_min(data, segment_ids, name=None):
    d, s = _t(data), _t(segment_ids)
    n = int(s.max()) + 1 if s.numel() else 0
    return _wrap(_reduce(d, s, n, "min"))


def send_u_recv(x, src_index, dst_index, reduce_op="sum", out_size=None, name=None):
    xt = _t(x)
    n = int(out_size) if out_size is not None and int(out_size) > 0 else xt.shape[0]
    msg = xt[_t(src_index).long()]
    return _wrap(_reduce(msg, _t(dst_index), n, reduce_op.lower()))


def send_ue_recv(x, y, src_index, dst_index, message_op="add", reduce_op="sum", out_size=None, name=None):
    xt, yt = _t(x), _t(y)
    n = int(out_size) if out_size is not None and int(out_size) > 0 else xt.shape[0]
    u = xt[_t(src_index).long()]
    ops = {"add": torch.add, "sub": torch.sub, "mul": torch.mul, "div": torch.div}
    msg = ops[message_op.lower()](u, yt)
    return _wrap(_reduce(msg, _t(dst_index), n, reduce_op.lower()))


def send_uv(x, y, src_index, dst_index, message_op="add", name=None):
    ops = {"add": torch.add, "sub": torch.sub, "mul": torch.mul, "div": torch.div}
    return _wrap(ops[message_op.lower()](_t(x)[_t(src_index).long()], _t(y)[_t(dst_index).long()]))


def reindex_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    """Relabel [x; neighbors] to consecutive ids (x first, then new nodes in first-seen order)."""
    xs = _t(x).cpu().numpy()
    nb = _t(neighbors).cpu().numpy()
    cnt = _t(count).cpu().numpy()
    mapping = {}
    for v in xs.tolist():
        mapping.setdefault(v, len(mapping))
    for v in nb.tolist():
        mapping.setdefault(v, len(mapping))
    src = np.array([mapping[v] for v in nb.tolist()], dtype=np.int64)
    dst = np.repeat(np.arange(len(xs), dtype=np.int64), cnt)
    nodes = np.array(list(mapping.keys()), dtype=xs.dtype)
    dev = _t(x).device
    return (_wrap(torch.from_numpy(src).to(dev)), _wrap(torch.from_numpy(dst).to(dev)),
            _wrap(torch.from_numpy(nodes).to(dev)))


def reindex_heter_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    """Heterogeneous reindex: one (neighbors, count) pair per edge type over the SAME centre nodes x; ids are
    shared across types (x first, then new neighbours in first-seen order over the concatenation) and the
    dst of each type repeats x by that type's counts. Reference: python/paddle/geometric/reindex.py."""
    nb = torch.cat([_t(n) for n in neighbors])
    src, _, nodes = reindex_graph(x, nb, torch.zeros(len(_t(x)), dtype=torch.int64))
    nx = len(_t(x))
    dst = torch.cat([torch.repeat_interleave(torch.arange(nx, dtype=torch.int64), _t(c).cpu().to(torch.int64))
                     for c in count]).to(_t(x).device)
    return src, _wrap(dst), nodes


def sample_neighbors(row, colptr, input_nodes, sample_size=-1, eids=None, return_eids=False, perm_buffer=None,
                     name=None):
    """CSC graph (row, colptr): sample up to sample_size in-neighbours per input node."""
    r = _t(row).cpu().numpy()
    cp = _t(colptr).cpu().numpy()
    nodes = _t(input_nodes).cpu().numpy()
    e = _t(eids).cpu().numpy() if eids is not None else None
    rng = np.random.default_rng()
    out, cnt, oe = [], [], []
    for v in nodes.tolist():
        lo, hi = int(cp[v]), int(cp[v + 1])
        idx = np.arange(lo, hi)
        if 0 <= sample_size < len(idx):
            idx = rng.choice(idx, sample_size, replace=False)
        out.append(r[idx])
        cnt.append(len(idx))
        if e is not None:
            oe.append(e[idx])
    dev = _t(row).device
    res = (_wrap(torch.from_numpy(np.concatenate(out) if out else np.zeros(0, r.dtype)).to(dev)),
           _wrap(torch.as_tensor(cnt, dtype=torch.int32, device=dev)))
    if return_eids:
        res = res + (_wrap(torch.from_numpy(np.concatenate(oe) if oe else np.zeros(0, np.int64)).to(dev)),)
    return res


def weighted_sample_neighbors(row, colptr, edge_weight, input_nodes, sample_size=-1, eids=None, return_eids=False,
                              name=None):
    r = _t(row).cpu().numpy()
    cp = _t(colptr).cpu().numpy()
    w = _t(edge_weight).cpu().numpy().astype(np.float64)
    nodes = _t(input_nodes).cpu().numpy()
    rng = np.random.default_rng()
    out, cnt = [], []
    for v in nodes.tolist():
        lo, hi = int(cp[v]), int(cp[v + 1])
        idx = np.arange(lo, hi)
        if 0 <= sample_size < len(idx):
            p = w[lo:hi] / w[lo:hi].sum()
            idx = rng.choice(idx, sample_size, replace=False, p=p)
        out.append(r[idx])
        cnt.append(len(idx))
    dev = _t(row).device
    return (_wrap(torch.from_numpy(np.concatenate(out) if out else np.zeros(0, r.dtype)).to(dev)),
            _wrap(torch.as_tensor(cnt, dtype=torch.int32, device=dev)))
