"""Data parallelism with bucketed, backward-overlapped gradient all-reduce over RCCL.

Reference: python/paddle/distributed/parallel.py:219 (DataParallel), paddle/fluid/distributed/collective/
reducer.cc (EagerReducer: buckets, ready-count, fused all-reduce).

MI355X design:
- every parameter's ``.grad`` is a view into a flat per-bucket buffer, so a ready bucket is
  all-reduced in place with no pack/unpack copies;
- buckets are planned in reverse registration order (≈ order grads become ready) by the native
  planner (``utils.native.plan_buckets``); the first-ready bucket is small (default 8 MB) so the first
  collective starts early, later buckets are large (default 64 MB) because xGMI ring all-reduce
  is latency-bound below a few MB and bandwidth-bound above;
- collectives are issued async (RCCL runs them on its own HIP stream ordered after the producing
  compute) and are all joined at the end of backward, before ``optimizer.step``;
- buckets are launched strictly in bucket-index order (reference reducer.cc:955 MarkGroupReady /
  next_group_): a bucket that fills early waits for its predecessors, so every rank issues the same
  collective sequence on the RCCL communicator even when grads become ready in a different order on
  different ranks (unused parameters, stream timing) — out-of-order all-reduces would hang RCCL;
- ReduceOp.AVG on RCCL (no extra scaling kernel); SUM + scale on gloo.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

from ..autograd.engine import queue_callback as _queue_callback
from ..distributed import collective as C
from ..framework.flags import flag
from ..framework.tensor import Tensor, _wrap
from ..nn.layer.layers import Layer
from ..utils import native


class _Bucket:
    __slots__ = ("params", "flat", "offsets", "pending", "work", "ready", "id")

    def __init__(self, params, dtype, device):
        self.params = params
        n = sum(p._t.numel() for p in params)
        self.flat = torch.zeros(n, dtype=dtype, device=device)
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += p._t.numel()
        self.pending = len(params)
        self.work = None
        self.ready = set()

    def view(self, i):
        p = self.params[i]
        o = self.offsets[i]
        return self.flat[o:o + p._t.numel()].view_as(p._t)


class DataParallel(Layer):
    def __init__(self, layers, strategy=None, comm_buffer_size=None, last_comm_buffer_size=8,
                 find_unused_parameters=False, group=None):
        super().__init__()
        self._layers = layers
        self.find_unused_parameters = find_unused_parameters
        self.group = group
        self._sync_enabled = True
        self._world = C.get_world_size(group)
        self._buckets = []
        self._param_loc = {}
        self._queued = False
        self._next_launch = 0  # position in _order of the next bucket to all-reduce
        self._order = []
        if self._world > 1:
            self._broadcast_params()
            self._build_buckets(comm_buffer_size, last_comm_buffer_size)

    # ------------------------------------------------------------------ setup
    def _broadcast_params(self):
        src = self.group.ranks[0] if self.group is not None else 0
        with torch.no_grad():
            for p in self._layers.parameters():
                dist.broadcast(p._t.data, src=src, group=C._pg(self.group))
            for b in self._layers.buffers():
                dist.broadcast(b._t.data, src=src, group=C._pg(self.group))

    def _build_buckets(self, comm_mb, last_mb):
        params = [p for p in self._layers.parameters() if not p.stop_gradient]
        # group by dtype/device (one flat buffer per bucket)
        by_key = {}
        for p in params:
            by_key.setdefault((p._t.dtype, p._t.device), []).append(p)
        # an explicit comm_buffer_size wins; otherwise FLAGS_dp_bucket_mb (sized for xGMI rings)
        mb = comm_mb if comm_mb is not None else flag("FLAGS_dp_bucket_mb", 128)
        for (dt, dev), ps in by_key.items():
            sizes = [p._t.numel() * p._t.element_size() for p in ps]
            # first-ready (last registered) bucket small, the rest large
            first = native.plan_buckets(sizes, int(last_mb * 2 ** 20))
            first_idx = first[0] if first else []
            rest = [i for i in range(len(ps)) if i not in set(first_idx)]
            plan = [first_idx]
            if rest:
                sub = native.plan_buckets([sizes[i] for i in rest], int(mb * 2 ** 20))
                plan += [[rest[j] for j in b] for b in sub]
            for idxs in plan:
                if not idxs:
                    continue
                b = _Bucket([ps[i] for i in idxs], dt, dev)
                bi = len(self._buckets)
                b.id = bi  # planned identity (the collective checker labels its all-reduce with it)
                self._buckets.append(b)
                for j, p in enumerate(b.params):
                    self._param_loc[id(p)] = (bi, j)
                    p._t.grad = b.view(j)
                    p._dp_bucket = (b, j)  # Optimizer.clear_grad keeps the bucket views (one memset per bucket)
                    p._t.register_post_accumulate_grad_hook(self._make_hook(p))
        # launch order across dtype groups by expected readiness: a bucket is complete when its earliest-registered
        # parameter gets its gradient, and backward reaches parameters in reverse registration order. Sorting by
        # that (stable, the same on every rank) interleaves the groups' buckets instead of holding every bucket of
        # the second group behind the first group's last one
        reg = {id(p): i for i, p in enumerate(params)}
        self._order = sorted(range(len(self._buckets)),
                             key=lambda bi: -min(reg[id(p)] for p in self._buckets[bi].params))

    def _make_hook(self, p):
        def hook(t):
            self._on_grad_ready(p)
        return hook

    # ------------------------------------------------------------------ comm
    def _on_grad_ready(self, p):
        if not self._sync_enabled or self._world == 1:
            return
        bi, j = self._param_loc[id(p)]
        b = self._buckets[bi]
        v = b.view(j)
        g = p._t.grad
        if g is None or g.data_ptr() != v.data_ptr():
            # grad was re-allocated (e.g. clear_grad(set_to_zero=False)): fold it back into the bucket
            if g is not None:
                v.copy_(g)
            p._t.grad = v
        if not self._queued:
            self._queued = True
            _queue_callback(self._finalize)
        if j in b.ready:
            return
        b.ready.add(j)
        if len(b.ready) == len(b.params):
            self._launch_ready()

    def _launch_ready(self):
        """Launch every full bucket at the head of the launch order (``_order``, by expected readiness)."""
        while self._next_launch < len(self._buckets):
            b = self._buckets[self._order[self._next_launch]]
            if b.work is not None or len(b.ready) < len(b.params):
                break
            self._launch(b)
            self._next_launch += 1

    def _launch(self, b):
        from ..distributed import collective_check as _cc
        pg = C._pg(self.group)
        with _cc.label(f"dp bucket {b.id}") if _cc.enabled() else contextlib.nullcontext():
            if dist.get_backend(pg) == "nccl":
                b.work = dist.all_reduce(b.flat, op=dist.ReduceOp.AVG, group=pg, async_op=True)
            else:
                b.flat.mul_(1.0 / self._world)
                b.work = dist.all_reduce(b.flat, op=dist.ReduceOp.SUM, group=pg, async_op=True)

    def _finalize(self):
        # the rest in bucket order; buckets with unused params keep those slices as they are (zero after
        # clear_grad) and are reduced like the others
        while self._next_launch < len(self._buckets):
            self._launch(self._buckets[self._order[self._next_launch]])
            self._next_launch += 1
        for b in self._buckets:
            b.work.wait()
            b.work = None
            b.ready = set()
        self._next_launch = 0
        self._queued = False
        from ..distributed import collective_check as _cc
        if _cc.enabled():
            _cc.check_collectives("DataParallel backward")

    # ------------------------------------------------------------------ api
    def forward(self, *inputs, **kwargs):
        return self._layers(*inputs, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def state_dict(self, *args, **kwargs):
        return self._layers.state_dict(*args, **kwargs)

    def set_state_dict(self, state_dict, use_structured_name=True):
        return self._layers.set_state_dict(state_dict, use_structured_name)

    set_dict = set_state_dict
    load_dict = set_state_dict

    def scale_loss(self, loss):
        return loss

    def apply_collective_grads(self):
        pass

    def parameters(self, include_sublayers=True):
        return self._layers.parameters(include_sublayers)

    def named_parameters(self, prefix="", include_sublayers=True, remove_duplicate=True):
        return self._layers.named_parameters(prefix, include_sublayers, remove_duplicate)
