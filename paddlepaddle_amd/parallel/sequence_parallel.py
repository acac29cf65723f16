"""Sequence parallelism with the tensor-parallel collectives overlapped by the GEMMs.

Reference: python/paddle/distributed/fleet/utils/sequence_parallel_utils.py:257 (SPInnerOverlapLinear: the dX
reduce-scatter of a column-parallel linear overlaps its dW GEMM), :429 ColumnSequenceParallelLinear, :564
RowSequenceParallelLinear; fleet/layers/mpu/mp_layers.py:190 (mp_async_allreduce).

Layout: between the tensor-parallel regions activations are TOKEN shards — the [B*S, H] token rows of a micro-
batch cut into mp contiguous blocks (rank r holds block r). LayerNorm, dropout, residual adds and the row-parallel
biases run on the shard; the mp collectives become all-gather / reduce-scatter of token blocks (half the bytes
of the all-reduce they replace) and each is hidden behind a GEMM on the RCCL stream:

  column-SP linear, forward : all-gather of the token blocks (async) || GEMM of this rank's own block; then
                              the other blocks' GEMMs as their rows have arrived.
  column-SP linear, backward: dX GEMM -> async reduce-scatter of dX || dW GEMM (+ bias/GELU gradients).
  row-SP linear, forward    : GEMM of the rows of block c, then an async reduce of that block to its owner c
                              || the GEMM of block c+1 (reduce-scatter pipelined over the blocks).
  row-SP linear, backward   : async all-gather of dY || dX / dW GEMMs of this rank's own block; then the rest.

On an 8 x MI355X node the TP pair talks over one direct xGMI link (no NVSwitch): a block is 1/mp of the
activation, so the transfer of one block hides behind the GEMM of another.

Parameters that see only a token shard (LayerNorm weights / biases, row-parallel biases, the position table)
carry ``sequence_parallel = True``; their gradients are partial over the mp group and are summed once per
optimizer step in one flat all-reduce (fleet HybridParallelOptimizer / the sharding engine), not per micro-batch.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import linear as _lin
from . import tensor_parallel as tp

# test hook: when a list, every collective issue / wait and every GEMM of the SP linears is appended in order
TRACE = None


def _log(*ev):
    if TRACE is not None:
        TRACE.append(ev)


def _ws(g):
    return tp._ws(g)


def _rank(g):
    return tp._rank(g)


def _pg(g):
    return g.process_group


def _blocks(x, n):
    return x.chunk(n, 0)


def all_gather_async(x, g, name="all_gather"):
    """(full, work): the token blocks of every rank concatenated in rank order, gathered asynchronously."""
    x = x.contiguous()
    full = torch.empty((x.shape[0] * _ws(g),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    work = dist.all_gather_into_tensor(full, x, group=_pg(g), async_op=True)
    _log("issue", name)
    return full, work


def reduce_scatter_async(x, g, name="reduce_scatter"):
    x = x.contiguous()
    out = torch.empty((x.shape[0] // _ws(g),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    work = dist.reduce_scatter_tensor(out, x, group=_pg(g), async_op=True)
    _log("issue", name)
    return out, work


def _wait(work, name):
    work.wait()
    _log("wait", name)


def _mm(x2, w):
    _log("gemm", tuple(x2.shape))
    return _lin._fwd_mm(x2, w)


class _ColumnSPLinear(torch.autograd.Function):
    """y[T, N/mp] = act(all_gather(x)[T, K] . w + b); x is this rank's token block [T/mp, K]."""

    @staticmethod
    def forward(ctx, x, w, b, act, group):
        n, r = _ws(group), _rank(group)
        x = x.contiguous()
        full, work = all_gather_async(x, group)
        gelu = act in ("gelu", "gelu_tanh", "gelu_approximate")
        ys, pres, bb = [None] * n, [None] * n, b
        order = [r] + [j for j in range(n) if j != r]  # own block first: it needs no communication
        for i, j in enumerate(order):
            if i == 1:
                _wait(work, "all_gather")
            xb = x if j == r else _blocks(full, n)[j]
            _log("gemm", tuple(xb.shape))
            if gelu:
                ys[j], pres[j], bb = _lin._fwd_bias_gelu(xb, w, b)
            else:
                ys[j] = _lin._fwd_mm(xb, w, b)
        if n == 1:
            _wait(work, "all_gather")
        y = torch.cat(ys, 0)
        ctx.gelu = gelu
        ctx.group = group
        ctx.bias = b
        ctx.has_b = b is not None
        if gelu:
            ctx.save_for_backward(full, w, bb, torch.cat(pres, 0))
        else:
            ctx.save_for_backward(full, w)
        ctx.w_leaf = _lin._leaf_weights(w)[0]
        return y

    @staticmethod
    def backward(ctx, dy):
        g = ctx.group
        if ctx.gelu:
            full, w, b, h = ctx.saved_tensors
        else:
            full, w = ctx.saved_tensors
        dy = dy.contiguous()
        if dy.dtype != full.dtype:
            dy = dy.to(full.dtype)
        db = None
        if ctx.gelu:
            dh, db = _bias_gelu_grad(h, b, dy, ctx.bias, ctx.needs_input_grad[2])
        else:
            dh = dy
            if ctx.has_b and ctx.needs_input_grad[2]:
                db = _bias_grad(dy, ctx.bias)
        # dX first, its reduce-scatter runs on the RCCL stream while the dW GEMM computes
        _log("gemm", "dgrad")
        dx_full = _lin._dgrad(dh, w)
        dx, work = reduce_scatter_async(dx_full, g)
        dw = None
        if ctx.needs_input_grad[1]:
            _log("gemm", "wgrad")
            dw = _wgrad_into(full, dh, w, wid=_lin._w_ident(w, ctx.w_leaf, True))
        _wait(work, "reduce_scatter")
        return dx, dw, db, None, None


class _ColumnSPLinearNT(torch.autograd.Function):
    """y[T, V/mp] = all_gather(x)[T, K] . w^T with w stored [V/mp, K] (the vocab-parallel LM head over the tied
    embedding table): the token all-gather overlaps the GEMM of this rank's own block; backward: dX GEMM, async
    reduce-scatter of dX (the vocab slices' partial input gradients) || dW GEMM."""

    @staticmethod
    def forward(ctx, x, w, group):
        n, r = _ws(group), _rank(group)
        x = x.contiguous()
        full, work = all_gather_async(x, group)
        ys = [None] * n
        order = [r] + [j for j in range(n) if j != r]
        for i, j in enumerate(order):
            if i == 1:
                _wait(work, "all_gather")
            xb = x if j == r else _blocks(full, n)[j]
            _log("gemm", tuple(xb.shape))
            ys[j] = _lin._nt_fwd(xb, w)
        ctx.group = group
        ctx.save_for_backward(full, w)
        return torch.cat(ys, 0)

    @staticmethod
    def backward(ctx, dy):
        full, w = ctx.saved_tensors
        dy = dy.contiguous()
        if dy.dtype != full.dtype:
            dy = dy.to(full.dtype)
        _log("gemm", "dgrad")
        dx_full = _lin._nt_dgrad(dy, w)
        dx, work = reduce_scatter_async(dx_full, ctx.group)
        dw = None
        if ctx.needs_input_grad[1]:
            _log("gemm", "wgrad")
            dw = _lin._nt_wgrad(dy, full)
        _wait(work, "reduce_scatter")
        return dx, dw, None


def column_sp_linear_nt(x, w, group=None):
    """Token block [T/mp, K] -> [T, V/mp] = all_gather(x) . w^T (w stored [V/mp, K])."""
    g = group or tp._mp_group()
    if _ws(g) == 1:
        return _lin.linear_nt(x, w)
    return _ColumnSPLinearNT.apply(x.reshape(-1, x.shape[-1]), w, g)


class _RowSPLinear(torch.autograd.Function):
    """y[T/mp, N] = reduce_scatter(x[T, K/mp] . w) (+ b, added by the caller on the shard)."""

    @staticmethod
    def forward(ctx, x, w, group):
        n, r = _ws(group), _rank(group)
        x = x.contiguous()
        ranks = group.ranks
        parts, works = [None] * n, []
        for c in range(n):  # same order on every rank: the reduces pair up
            yc = _mm(_blocks(x, n)[c], w).contiguous()
            parts[c] = yc
            if n > 1:
                works.append(dist.reduce(yc, dst=ranks[c], op=dist.ReduceOp.SUM, group=_pg(group), async_op=True))
                _log("issue", "reduce")
        for wk in works:
            _wait(wk, "reduce")
        ctx.group = group
        ctx.save_for_backward(x, w)
        ctx.w_leaf = _lin._leaf_weights(w)[0]
        return parts[r]

    @staticmethod
    def backward(ctx, dy):
        g = ctx.group
        n, r = _ws(g), _rank(g)
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        full, work = all_gather_async(dy, g)
        xb = _blocks(x, n)
        dxs = [None] * n
        dw = None
        order = [r] + [j for j in range(n) if j != r]
        for i, j in enumerate(order):
            if i == 1:
                _wait(work, "all_gather")
            dyj = dy if j == r else _blocks(full, n)[j]
            if ctx.needs_input_grad[0]:
                _log("gemm", "dgrad")
                dxs[j] = _lin._dgrad(dyj, w)
            if ctx.needs_input_grad[1]:
                _log("gemm", "wgrad")
                dw = _wgrad_into(xb[j], dyj, w, dw, last=(i == n - 1),
                                 wid=_lin._w_ident(w, ctx.w_leaf, True))
        if n == 1:
            _wait(work, "all_gather")
        dx = torch.cat(dxs, 0) if ctx.needs_input_grad[0] else None
        return dx, dw, None


def _bias_grad(dy, bias):
    mg = _lin._vector_main_grad(bias, dy.dtype)
    if mg is not None:  # added straight into the flat grad buffer
        _lin.colsum(dy, acc=mg[0])
        mg[1](bias)
        return None
    return _lin.colsum(dy)


def _bias_gelu_grad(h, b, dy, bias, need_db):
    from ..ops import _loader as L
    rows, cols = h.shape
    if L.hip_enabled_for(h) and L.has("pa_bias_gelu_bwd") and cols % 8 == 0:
        dh = torch.empty_like(h)
        mg = _lin._vector_main_grad(bias, b.dtype) if need_db else None
        db = mg[0] if mg is not None else torch.empty(cols, dtype=b.dtype, device=b.device)
        ws = torch.empty(256 * cols, dtype=torch.float32, device=h.device)
        L.call("pa_bias_gelu_bwd", L.ptr(h), L.ptr(b), L.ptr(dy), L.ptr(dh), L.ptr(db), L.ptr(ws), rows, cols,
               L.dcode(h) | ((mg is not None) << 8), L.stream_ptr())
        if mg is not None:
            mg[1](bias)
            db = None
        return dh, (db if need_db else None)
    # generic path: h is the pre-activation without the bias (bb == b) or with it (bb == 0)
    hb = (h.float() + b.float()).requires_grad_(True)
    with torch.enable_grad():
        y = torch.nn.functional.gelu(hb, approximate="tanh")
        (dh,) = torch.autograd.grad(y, hb, dy.float())
    dh = dh.to(h.dtype)
    return dh, (dh.float().sum(0).to(b.dtype) if need_db else None)


def _wgrad_into(x2, dy2, w, acc=None, last=True, wid=None):
    """x2^T dy2 for weight ``w``: into its main-grad buffer when registered (the engine's grad-ready handler runs
    after the last block), else a fresh dW / accumulated into ``acc``. ``wid``: the parameter ``w`` stands for
    (ops/linear.py _w_ident: a recompute hands saved weights back detached)."""
    w = w if wid is None else wid
    ent = _lin._main_grad_of(w)
    if ent is not None and ent[1].dtype == dy2.dtype:
        _, buf, on_ready = ent
        _lin._wgrad(x2, dy2, acc=buf)
        if last:
            on_ready(w)
        return None
    if acc is None:
        return _lin._wgrad(x2, dy2)
    return _lin._wgrad(x2, dy2, acc=acc)


def column_sp_linear(x, w, b=None, act=None, group=None):
    """Token block [T/mp, ..., K] -> [T, ..., N/mp] (column-parallel weights; blocks split along dim 0)."""
    g = group or tp._mp_group()
    if _ws(g) == 1:
        return _lin.fused_linear(x, w, b, act=act)
    lead = x.shape[:-1]
    y = _ColumnSPLinear.apply(x.reshape(-1, x.shape[-1]), w, b, act, g)
    return y.view((lead[0] * _ws(g),) + tuple(lead[1:]) + (w.shape[1],))


def row_sp_linear(x, w, group=None):
    """[T, ..., K/mp] (row-parallel weights) -> this rank's token block [T/mp, ..., N] of the mp-summed product."""
    g = group or tp._mp_group()
    if _ws(g) == 1:
        return _lin.fused_linear(x, w, None)
    lead = x.shape[:-1]
    y = _RowSPLinear.apply(x.reshape(-1, x.shape[-1]), w, g)
    return y.view((lead[0] // _ws(g),) + tuple(lead[1:]) + (w.shape[1],))


class _SPAllGather(torch.autograd.Function):
    """Token blocks -> all tokens; backward: reduce-scatter (partial gradients of the consumer are summed)."""

    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        full, work = all_gather_async(x, g, "all_gather_sync")
        _wait(work, "all_gather_sync")
        return full

    @staticmethod
    def backward(ctx, d):
        out, work = reduce_scatter_async(d, ctx.g, "reduce_scatter_sync")
        _wait(work, "reduce_scatter_sync")
        return out, None


class _SPReduceScatter(torch.autograd.Function):
    """Partial sums over all tokens -> this rank's token block of the sum; backward: all-gather."""

    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        out, work = reduce_scatter_async(x, g, "reduce_scatter_sync")
        _wait(work, "reduce_scatter_sync")
        return out

    @staticmethod
    def backward(ctx, d):
        full, work = all_gather_async(d, ctx.g, "all_gather_sync")
        _wait(work, "all_gather_sync")
        return full, None


def gather_tokens(x, group=None):
    g = group or tp._mp_group()
    return x if _ws(g) == 1 else _SPAllGather.apply(x, g)


def reduce_scatter_tokens(x, group=None):
    g = group or tp._mp_group()
    return x if _ws(g) == 1 else _SPReduceScatter.apply(x, g)


def scatter_tokens(x, group=None):
    """This rank's block of replicated token rows (no communication; backward all-gathers)."""
    g = group or tp._mp_group()
    if _ws(g) == 1:
        return x
    from ..distributed.fleet.utils.sequence_parallel_utils import _Scatter
    return _Scatter.apply(x, g)


def token_block_range(T, group=None):
    g = group or tp._mp_group()
    n, r = _ws(g), _rank(g)
    per = T // n
    return r * per, (r + 1) * per


def mark_sequence_parallel(*params):
    for p in params:
        if p is not None:
            p.sequence_parallel = True


def allreduce_sequence_parallel_grads(params, group):
    """Sum the partial gradients of sequence-parallel parameters over the mp group: ONE flat all-reduce for all
    of them (once per optimizer step: gradient accumulation is linear)."""
    if group is None or _ws(group) == 1:
        return
    gs = [p._t.grad for p in params if getattr(p, "sequence_parallel", False) and p._t.grad is not None
          and not getattr(p, "_sp_hooked", False)]
    if not gs:
        return
    flat = torch.cat([g.reshape(-1).float() for g in gs])
    dist.all_reduce(flat, group=_pg(group))
    off = 0
    for g in gs:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n
