"""ZeRO-style sharded data parallelism (Fleet sharding stage 1 / 2 / 3) over RCCL.

Reference: python/paddle/distributed/sharding/group_sharded.py:50 (group_sharded_parallel),
fleet/meta_parallel/sharding/group_sharded_stage2.py:47, group_sharded_optimizer_stage2.py:53,
group_sharded_stage3.py:85 (forward pre/post hooks gather & release params, backward hooks
reduce-scatter grads, optimizer steps on the local shard).

MI355X-native design (one process per GPU, flat buffers, no per-parameter collectives):
* Parameters are grouped into *units* (each block of a LayerList = one unit, everything else = the
  root unit) and, inside a unit, into flat buffers by (dtype, weight-decay). A flat buffer is padded
  to a multiple of the sharding degree W; rank r owns elements [r*S, (r+1)*S).
* Every model parameter's storage is a view into its unit's full flat buffer, and every gradient is a
  view into the unit's full flat grad buffer, so a collective moves one contiguous buffer per unit.
* Gradients are reduce-scattered per unit as soon as the unit's backward is done (overlaps with the
  remaining backward), in bf16, and accumulated into an fp32 shard gradient (gradient accumulation
  safe). The optimizer runs only on the local shards (fused multi-tensor AdamW with fp32 master
  shard). Stage 1/2 then all-gather the updated shards back into the replicated flat params.
* Stage 3 additionally frees each unit's full parameter storage after use (forward post-hook;
  re-gathered by a pre-backward hook on the unit output) and prefetches the next unit's all-gather on
  RCCL's stream while the current unit computes. With 288 GB HBM per GPU, units are whole
  transformer blocks (a 13B block is 630 MB in bf16) — few, large collectives that keep the xGMI
  rings in their bandwidth-bound regime.
* ``offload=True`` (reference group_sharded_stage3.py:98-127 keeps fp32 master weights and the optimizer
  update on the CPU): here the optimizer state of the local shards (fp32 master weights, moments) lives in
  pinned host memory between steps and is streamed through the GPU one unit at a time — H2D of unit i+1 on
  a copy stream overlaps the fused AdamW update of unit i, whose state goes back D2H behind it — so HBM
  holds the state of at most two units (instead of 12 bytes per local parameter) and the update still runs
  on the MFMA-free, bandwidth-bound HIP kernel rather than on host cores.
"""
from __future__ import annotations

import contextlib

import os

import torch
import torch.distributed as dist

from ..autograd.engine import queue_callback as _queue_callback, register_grad_hook as _register_grad_hook
from ..distributed import collective as C
from ..framework.tensor import Parameter, Tensor, _wrap
from ..nn.layer.common import LayerList
from ..nn.layer.layers import Layer


def _is_nccl(pg):
    return dist.get_backend(pg) == "nccl"


# biases / norm parameters accumulate in the HIP finalize kernels too (PADDLE_AMD_VECTOR_MAIN_GRAD=0: through autograd)
_VECTOR_MAIN_GRAD = os.environ.get("PADDLE_AMD_VECTOR_MAIN_GRAD", "1") != "0"


class _Flat:
    """One flat buffer of same-dtype, same-decay parameters of a unit."""

    def __init__(self, params, world, rank, decay, distributed=False):
        self.params = params
        self.world, self.rank = world, rank
        self.decay = decay
        self.distributed = distributed  # tensor-parallel shards (differ across the mp group)
        t0 = params[0]._t
        self.dtype, self.device = t0.dtype, t0.device
        self.numels = [p._t.numel() for p in params]
        total = sum(self.numels)
        self.shard_size = (total + world - 1) // world
        self.padded = self.shard_size * world
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        full = torch.zeros(self.padded, dtype=self.dtype, device=self.device)
        with torch.no_grad():
            for p, o, n in zip(params, self.offsets, self.numels):
                full[o:o + n].copy_(p._t.detach().reshape(-1))
        self.full = full
        # alias over the same storage with its own version counter: collectives write through it so
        # re-gathering (stage 3) does not bump the version of tensors autograd saved in forward
        self.gbuf = torch.empty(0, dtype=self.dtype, device=self.device).set_(full.untyped_storage(), 0,
                                                                             (self.padded,))
        # local shard as an optimizer-visible Parameter (trainable flat view of my slice)
        sh = full[rank * self.shard_size:(rank + 1) * self.shard_size].detach()
        if world > 1:
            sh = sh.clone()
        # degree 1: the shard IS the full buffer and grads stay in the flat bf16 grad buffer
        self.shard = Parameter(sh, trainable=True, name=f"sharded_flat_{id(self)}")
        self.shard.need_clip = True
        self.shard.is_distributed = distributed
        if world > 1 and sh.dtype != torch.float32 and hasattr(self.shard._t, "grad_dtype"):
            self.shard._t.grad_dtype = None  # bf16 shard, fp32 reduce-scattered gradient
        self.shard_grad = torch.zeros(self.shard_size, dtype=torch.float32, device=self.device) if world > 1 else None
        self.full_grad = None
        self.ready_fn = None  # engine's grad-ready handler (set once the unit is built)
        # re-point model params at views of the full buffer
        for p, o, n in zip(params, self.offsets, self.numels):
            req = p._t.requires_grad
            p._t = full[o:o + n].view(p._t.shape).detach().requires_grad_(req)

    # -- grads
    def alloc_full_grad(self):
        if self.full_grad is None:
            from ..ops.linear import register_main_grad
            self.full_grad = torch.zeros(self.padded, dtype=self.dtype, device=self.device)
            for p, o, n in zip(self.params, self.offsets, self.numels):
                view = self.full_grad[o:o + n].view(p._t.shape)
                p._t.grad = view
                if self.ready_fn is not None and (p._t.dim() == 2 or _VECTOR_MAIN_GRAD):
                    # linear weights: the wgrad GEMM accumulates into this view directly; biases and norm
                    # parameters: the HIP gradient-finalize kernels add into it (no autograd accumulation pass)
                    register_main_grad(p._t, view, self.ready_fn)
        return self.full_grad

    def fold_param_grads(self):
        """Make sure every param grad lives in full_grad (autograd may have replaced a .grad)."""
        fg = self.alloc_full_grad()
        for p, o, n in zip(self.params, self.offsets, self.numels):
            g = p._t.grad
            v = fg[o:o + n]
            if g is None:
                continue
            if g.data_ptr() != v.data_ptr():
                v.copy_(g.reshape(-1))
                p._t.grad = v.view(p._t.shape)

    def drop_full_grad(self):
        from ..ops.linear import unregister_main_grad
        for p in self.params:
            p._t.grad = None
            unregister_main_grad(p._t)
        self.full_grad = None

    # -- params (stage 3 storage management)
    def free_full(self):
        self.full.untyped_storage().resize_(0)

    def alloc_full(self):
        st = self.full.untyped_storage()
        need = self.padded * self.full.element_size()
        if st.size() != need:
            st.resize_(need)


class _Unit:
    def __init__(self, name, layer, params, world, rank, decay_fn):
        self.name = name
        self.layer = layer
        self.flats = []
        groups = {}
        for p in params:
            key = (p._t.dtype, bool(decay_fn(p)), bool(getattr(p, "is_distributed", False)),
                   bool(getattr(p, "sequence_parallel", False)))
            groups.setdefault(key, []).append(p)
        for (dt, dec, dist_, sp), ps in groups.items():
            f = _Flat(ps, world, rank, dec, dist_)
            f.sequence_parallel = sp  # grads partial over the mp group (token-block inputs)
            self.flats.append(f)
        self.n_params = len(params)
        self.ready = set()
        self.gathered = True
        self.gather_work = []
        self.rs_work = []
        self.rs_tmp = []
        self.id_set = {id(p) for p in params}


class GroupShardedEngine:
    """Implements stage 1/2/3 over a model + inner optimizer."""

    def __init__(self, model, optimizer, stage, group=None, decay_fn=None, mp_group=None, dp_group=None,
                 keep_params=None, pp_group=None, offload=False, sep_group=None):
        self.model = model
        self.offload = bool(offload)
        self._copy_stream = None
        self.stage = stage
        self.group = group
        self.pg = C._pg(group)
        # hybrid composition (reference: dygraph_sharding_optimizer.py:54 takes hcg's sharding group;
        # group_sharded_stage3.py:85 dp_group): tensor-parallel shards live in the mp group, an outer
        # data-parallel group (replicas of the sharded state) averages the shard gradients
        self.mp_group = mp_group if (mp_group is not None and getattr(mp_group, "nranks", 1) > 1) else None
        self.dp_group = dp_group if (dp_group is not None and getattr(dp_group, "nranks", 1) > 1) else None
        self.pp_group = pp_group if (pp_group is not None and getattr(pp_group, "nranks", 1) > 1) else None
        # segment parallel (sep): the sep ranks hold the same shards for different sequence segments, so their
        # shard gradients are summed over the sep group (reference: sep gradients are not averaged)
        self.sep_group = sep_group if (sep_group is not None and getattr(sep_group, "nranks", 1) > 1) else None
        self._keep_override = keep_params
        self.world = C.get_world_size(group)
        self.rank = C.get_rank(group) if group is not None else (dist.get_rank() if dist.is_initialized() else 0)
        self.inner_opt = optimizer
        if decay_fn is None:
            fn = getattr(optimizer, "_apply_decay_param_fun", None)
            decay_fn = (lambda p: fn(p.name)) if fn is not None else (lambda p: True)
        self._broadcast_params()
        self.units = self._build_units(decay_fn)
        self._flat_by_param = {}
        for u in self.units:
            for f in u.flats:
                for p in f.params:
                    self._flat_by_param[id(p)] = (u, f)
        self._queued = False
        self._in_backward = False
        self._sync = True
        self.keep_params = self._decide_keep_params()
        self._install_hooks()
        self._rebind_optimizer(optimizer)
        if stage == 3:
            for u in self.units[1:]:
                self._release(u)

    def _decide_keep_params(self):
        """Stage 3 on a 288 GB MI355X: when the full bf16 parameters + gradients take a modest share of
        HBM, keep each unit's gathered parameters resident from its first all-gather until the
        optimizer step (ZeRO-3 "live parameters"), instead of re-gathering twice per micro-batch.
        Per step that is one all-gather + one reduce-scatter of the model instead of 3 x accum."""
        if self.stage != 3 or self.world == 1:
            return False
        if self._keep_override is not None:
            return bool(self._keep_override)
        from ..framework.flags import flag
        mode = str(flag("FLAGS_sharding_stage3_keep_params", "auto")).lower()
        if mode in ("0", "false", "off"):
            return False
        if mode in ("1", "true", "on"):
            return True
        nbytes = sum(f.padded * f.full.element_size() for u in self.units for f in u.flats)
        dev = self.units[0].flats[0].device if self.units else torch.device("cpu")
        if dev.type != "cuda":
            return False
        total = torch.cuda.get_device_properties(dev).total_memory
        return 2 * nbytes < 0.35 * total

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient-accumulation micro-batches: grads accumulate locally, no reduce-scatter."""
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    # ------------------------------------------------------------------ construction
    def _broadcast_params(self):
        with torch.no_grad():
            if self.world > 1:
                src = self.group.ranks[0] if self.group is not None else 0
                for p in self.model.parameters():
                    dist.broadcast(p._t.data, src=src, group=self.pg)
            for og in (self.dp_group, self.sep_group):  # replicas of the sharded state start identical
                if og is not None:
                    for p in self.model.parameters():
                        dist.broadcast(p._t.data, src=og.ranks[0], group=og.process_group)

    def _build_units(self, decay_fn):
        unit_layers = []
        seen = set()
        for _, l in self.model.named_sublayers(include_self=True):
            if isinstance(l, LayerList):
                for child in l:
                    unit_layers.append(child)
        units = []
        claimed = set()
        for i, l in enumerate(unit_layers):
            ps = [p for p in l.parameters() if not p.stop_gradient and id(p) not in claimed]
            if not ps:
                continue
            claimed.update(id(p) for p in ps)
            units.append((f"unit{i}", l, ps))
        root_ps = [p for p in self.model.parameters() if not p.stop_gradient and id(p) not in claimed]
        out = []
        if root_ps:
            out.append(_Unit("root", self.model, root_ps, self.world, self.rank, decay_fn))
        for name, l, ps in units:
            out.append(_Unit(name, l, ps, self.world, self.rank, decay_fn))
        return out

    def _rebind_optimizer(self, opt):
        shards = []
        decay_ids = set()
        for u in self.units:
            for f in u.flats:
                shards.append(f.shard)
                if f.decay:
                    decay_ids.add(f.shard.name)
        opt._param_groups = [{"params": shards}]
        opt._parameter_list = shards
        if hasattr(opt, "_apply_decay_param_fun"):
            opt._apply_decay_param_fun = (lambda n, _d=decay_ids: n in _d)
        clip = getattr(opt, "_grad_clip", None)
        if clip is not None and hasattr(clip, "_extra_sq_norm_fn") and (
                self.world > 1 or self.mp_group is not None or self.pp_group is not None):
            pg, shard_sum = self.pg, self.world > 1  # pg None = the default (world) group
            mp_pg = self.mp_group.process_group if self.mp_group is not None else None
            pp_pg = self.pp_group.process_group if self.pp_group is not None else None

            def _param_sq(params):
                # shards partition each flat over the sharding group (sum there); tensor-parallel flats
                # are also disjoint across the mp group (sum there), replicated flats are counted once
                from ..ops.optim import global_sq_norm
                dev = params[0]._t.device
                dg = [p._t.grad for p in params if getattr(p, "is_distributed", False)]
                rg = [p._t.grad for p in params if not getattr(p, "is_distributed", False)]
                sq_d = (global_sq_norm(dg) if dg else torch.zeros((), device=dev)).float().reshape(1).clone()
                sq_r = (global_sq_norm(rg) if rg else torch.zeros((), device=dev)).float().reshape(1)
                if mp_pg is not None:
                    dist.all_reduce(sq_d, group=mp_pg)
                sq = sq_d + sq_r
                if shard_sum:
                    dist.all_reduce(sq, group=pg)
                if pp_pg is not None:  # pipeline stages hold disjoint layers
                    dist.all_reduce(sq, group=pp_pg)
                return sq[0]
            clip._param_sq_fn = _param_sq
            if mp_pg is None and pp_pg is None and shard_sum:  # optimizers that clip through _global_norm
                def _allreduce_sq(sq):
                    dist.all_reduce(sq, group=pg)
                    return sq
                clip._extra_sq_norm_fn = _allreduce_sq

    # ------------------------------------------------------------------ hooks
    def _install_hooks(self):
        for ui, u in enumerate(self.units):
            hook = self._make_grad_hook(u)
            for f in u.flats:
                f.ready_fn = hook
                for p in f.params:
                    p._t.register_post_accumulate_grad_hook(hook)
            if ui == 0:
                continue  # root unit: gathered for the whole step (embedding / tied head / final norm)
            u.layer.register_forward_pre_hook(self._make_fwd_pre(ui))
            u.layer.register_forward_post_hook(self._make_fwd_post(ui))

    def _make_fwd_pre(self, ui):
        def hook(layer, inputs):
            u = self.units[ui]
            self._gather(u)
            self._wait_gather(u)
            if self.stage == 3 and torch.is_grad_enabled() and ui + 1 < len(self.units):
                self._gather(self.units[ui + 1])  # prefetch next block
            return None
        return hook

    def _make_fwd_post(self, ui):
        def hook(layer, inputs, out):
            u = self.units[ui]
            if torch.is_grad_enabled():
                t = out._t if isinstance(out, Tensor) else None
                if t is not None and t.requires_grad:
                    _register_grad_hook(t, self._make_pre_backward(ui))
            if self.stage == 3 and not self._in_backward and not self.keep_params:
                self._release(u)
            return None
        return hook

    def _make_pre_backward(self, ui):
        def hook(g):
            self._in_backward = True
            self._queue_finalize()
            u = self.units[ui]
            self._gather(u)
            self._wait_gather(u)
            for f in u.flats:
                f.alloc_full_grad()  # grads accumulate in place into the unit's flat grad buffer
            if self.stage == 3 and ui - 1 >= 1:
                self._gather(self.units[ui - 1])
            return None
        return hook

    def _make_grad_hook(self, u):
        def hook(t):
            self._queue_finalize()
            u.ready.add(id(t))
            if not self._sync:
                return  # accumulation micro-batch: grads stay in the unit's flat grad buffer
            # root unit (tied embedding used twice) is flushed at the end of backward instead
            if u is not self.units[0] and len(u.ready) == u.n_params:
                self._reduce_scatter(u)
                if self.stage == 3 and not self.keep_params:
                    self._release(u)
        return hook

    def _queue_finalize(self):
        if not self._queued:
            self._queued = True
            _queue_callback(self._finalize_backward)

    # ------------------------------------------------------------------ collectives
    def _gather(self, u):
        from ..distributed import collective_check as _cc
        if _cc.enabled() and not (u.gathered or self.world == 1):
            with _cc.label(f"ag unit {self.units.index(u)}"):
                return self._gather_impl(u)
        return self._gather_impl(u)

    def _gather_impl(self, u):
        if u.gathered or self.world == 1:
            u.gathered = True
            return
        for f in u.flats:
            f.alloc_full()
            out = f.gbuf
            inp = f.shard._t.detach()
            if inp.dtype != out.dtype:
                inp = inp.to(out.dtype)
            u.gather_work.append(dist.all_gather_into_tensor(out, inp, group=self.pg, async_op=True))
        u.gathered = True

    def _wait_gather(self, u):
        for w in u.gather_work:
            w.wait()
        u.gather_work = []

    def _release(self, u):
        if self.stage != 3 or self.world == 1:
            return
        self._wait_gather(u)
        for f in u.flats:
            f.free_full()
        u.gathered = False

    def _reduce_scatter(self, u):
        from ..distributed import collective_check as _cc
        if _cc.enabled():
            with _cc.label(f"rs unit {self.units.index(u)}"):
                return self._reduce_scatter_impl(u)
        return self._reduce_scatter_impl(u)

    def _reduce_scatter_impl(self, u):
        for f in u.flats:
            f.fold_param_grads()
            fg = f.full_grad
            if self.world == 1:
                continue  # grads stay (and accumulate) in the flat buffer
            tmp = torch.empty(f.shard_size, dtype=fg.dtype, device=fg.device)
            if _is_nccl(self.pg):
                w = dist.reduce_scatter_tensor(tmp, fg, op=dist.ReduceOp.AVG, group=self.pg, async_op=True)
            else:
                fg.mul_(1.0 / self.world)
                w = dist.reduce_scatter_tensor(tmp, fg, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            u.rs_work.append(w)
            u.rs_tmp.append((f, tmp))
        u.ready = set()

    def _finalize_backward(self):
        if not self._sync:
            for u in self.units:
                u.ready = set()
                if self.stage == 3 and u is not self.units[0] and not self.keep_params:
                    self._release(u)
            self._queued = False
            self._in_backward = False
            return
        # flush units whose grads were never (fully) produced, then join every reduce-scatter
        for u in self.units:
            if u.ready or (not u.rs_tmp and any(f.full_grad is not None for f in u.flats)):
                self._reduce_scatter(u)
        for u in self.units:
            for w in u.rs_work:
                w.wait()
            for f, tmp in u.rs_tmp:
                f.shard_grad.add_(tmp.float())
                f.drop_full_grad()
            u.rs_work, u.rs_tmp = [], []
            if self.world == 1:
                continue
            if self.stage == 3 and u is not self.units[0]:
                if not self.keep_params:
                    self._release(u)
            else:
                for f in u.flats:
                    if f.full_grad is not None:
                        f.drop_full_grad()
        self._queued = False
        self._in_backward = False

    # ------------------------------------------------------------------ optimizer
    @torch.no_grad()
    def step(self):
        from ..distributed import collective_check as _cc
        if _cc.enabled():
            _cc.check_collectives("sharding step")
        dp_work = []
        sp_mp = self.mp_group is not None
        sp = []
        for u in self.units:
            for f in u.flats:
                if self.world == 1:
                    f.shard._t.grad = f.alloc_full_grad()
                else:
                    f.shard._t.grad = f.shard_grad
                if sp_mp and getattr(f, "sequence_parallel", False):
                    sp.append(f.shard._t.grad)  # reduced below as one flat over mp, then dp
                    continue
                if self.sep_group is not None:  # summed over the sequence segments before the dp average
                    dist.all_reduce(f.shard._t.grad, group=self.sep_group.process_group)
                if self.dp_group is not None:  # replicas of this shard: average across the outer dp group
                    g = f.shard._t.grad
                    g.mul_(1.0 / self.dp_group.nranks)
                    dp_work.append(dist.all_reduce(g, group=self.dp_group.process_group, async_op=True))
        if sp:
            # sequence-parallel flats (LayerNorm / row-parallel bias / position table): each mp rank holds the
            # gradient of its own token blocks. One flat holds all of them: summed over the mp group first, then
            # averaged over the dp replicas; the per-flat dp all-reduces above skip these grads, so no collective
            # ever reads a buffer another one is still writing.
            flat = torch.cat([g.reshape(-1).float() for g in sp])
            dist.all_reduce(flat, group=self.mp_group.process_group)
            if self.sep_group is not None:
                dist.all_reduce(flat, group=self.sep_group.process_group)
            if self.dp_group is not None:
                flat.mul_(1.0 / self.dp_group.nranks)
                dp_work.append(dist.all_reduce(flat, group=self.dp_group.process_group, async_op=True))
        for w in dp_work:
            w.wait()
        if sp:
            off = 0
            for g in sp:
                g.copy_(flat[off:off + g.numel()].view_as(g))
                off += g.numel()
        if self.offload:
            self._offload_step()
        else:
            self.inner_opt.step()
        if self.world == 1:
            return  # shard aliases the full buffer: nothing to publish
        for u in self.units:
            if self.stage == 3 and u is not self.units[0]:
                if self.keep_params:
                    u.gathered = False  # stale after the update; storage kept, re-filled on next use
                continue
            for f in u.flats:
                dist.all_gather_into_tensor(f.gbuf, f.shard._t.detach().to(f.full.dtype), group=self.pg)

    # ------------------------------------------------------------------ offload
    def _state_slots(self, p):
        """(dict, key) of every optimizer-state tensor of shard ``p`` (accumulators + master weight)."""
        opt = self.inner_opt
        out = [(d, id(p)) for d in opt._accumulators.values() if id(p) in d]
        if id(p) in opt._master_weights:
            out.append((opt._master_weights, id(p)))
        return out

    @staticmethod
    def _host_copy(t):
        return torch.empty(t.shape, dtype=t.dtype, pin_memory=True)

    def _swap_in(self, shards, dev):
        """Start the H2D copies of ``shards``' host state on the copy stream; returns the ready event."""
        if dev.type != "cuda":  # CPU tensors: the state already lives in host memory
            return None
        cs = self._copy_stream
        cs.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(cs):
            for p in shards:
                for d, k in self._state_slots(p):
                    h = d[k]
                    if h.device.type == "cpu":
                        g = torch.empty(h.shape, dtype=h.dtype, device=dev)
                        g.copy_(h, non_blocking=True)
                        g._pa_host = h
                        d[k] = g
        ev = torch.cuda.Event()
        ev.record(cs)
        return ev

    def _swap_out(self, shards, dev):
        """Queue the D2H copies of the updated state behind the update, then point the optimizer at the host
        tensors; the device buffers go back to the allocator once the copy stream has read them."""
        if dev.type != "cuda":
            return
        cs = self._copy_stream
        cs.wait_stream(torch.cuda.current_stream(dev))
        bufs = []
        with torch.cuda.stream(cs):
            for p in shards:
                for d, k in self._state_slots(p):
                    g = d[k]
                    if g.device.type == "cpu":
                        continue
                    h = getattr(g, "_pa_host", None)
                    if h is None:
                        h = self._host_copy(g)
                    h.copy_(g, non_blocking=True)
                    g.record_stream(cs)
                    bufs.append(g)
                    d[k] = h
        ev = torch.cuda.Event()
        ev.record(cs)
        # the device buffers are released one unit later, after the compute stream has waited for their
        # copies (allocators that ignore record_stream stay safe; at most ~2 units of state stay in HBM)
        if self._inflight:
            pev, _ = self._inflight.pop(0)
            torch.cuda.current_stream(dev).wait_event(pev)
        self._inflight.append((ev, bufs))

    @torch.no_grad()
    def _offload_step(self):
        """Optimizer.step (optimizer.py:189) unit by unit with the state streamed from pinned host memory."""
        from ..ops.linear import bump_weight_epoch
        opt = self.inner_opt
        bump_weight_epoch()
        opt._step_count += 1
        opt._apply_clip()
        group = opt._param_groups[0]
        chunks = [[f.shard for f in u.flats if f.shard._t.grad is not None] for u in self.units]
        chunks = [c for c in chunks if c]
        if not chunks:
            return
        dev = chunks[0][0]._t.device
        if dev.type == "cuda" and self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(dev)
        self._inflight = []
        ev = self._swap_in(chunks[0], dev)
        for i, ps in enumerate(chunks):
            nxt = self._swap_in(chunks[i + 1], dev) if i + 1 < len(chunks) else None
            if ev is not None:
                torch.cuda.current_stream(dev).wait_event(ev)
            opt._update_group(group, ps)
            self._swap_out(ps, dev)
            ev = nxt
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).wait_stream(self._copy_stream)
        self._inflight = []

    def offloaded_bytes(self):
        """Bytes of optimizer state currently held in host memory."""
        tot = 0
        for u in self.units:
            for f in u.flats:
                for d, k in self._state_slots(f.shard):
                    if d[k].device.type == "cpu":
                        tot += d[k].numel() * d[k].element_size()
        return tot

    def clear_grad(self, set_to_zero=True):
        for u in self.units:
            for f in u.flats:
                if self.world == 1:
                    if f.full_grad is not None:
                        f.full_grad.zero_()
                else:
                    f.shard_grad.zero_()
                f.shard._t.grad = None

    def pre_forward(self):
        """Root unit (embeddings / tied head / final norm) is gathered for the whole step."""
        if not self.units:
            return
        self._gather(self.units[0])
        self._wait_gather(self.units[0])
        if torch.is_grad_enabled():
            for f in self.units[0].flats:
                f.alloc_full_grad()

    @torch.no_grad()
    def reshard_from_full(self):
        for u in self.units:
            for f in u.flats:
                f.shard._t.data.copy_(f.full[f.rank * f.shard_size:(f.rank + 1) * f.shard_size])

    @torch.no_grad()
    def gather_all(self):
        """Materialise every full parameter (for state_dict / eval under stage 3)."""
        for u in self.units:
            self._gather(u)
            self._wait_gather(u)


class GroupShardedModel(Layer):
    def __init__(self, engine):
        super().__init__()
        object.__setattr__(self, "_engine", engine)
        self._layers = engine.model

    def forward(self, *args, **kwargs):
        self._engine.pre_forward()
        return self._layers(*args, **kwargs)

    def no_sync(self):
        return self._engine.no_sync()

    def state_dict(self, *args, **kwargs):
        self._engine.gather_all()
        return self._layers.state_dict(*args, **kwargs)

    def set_state_dict(self, sd, use_structured_name=True):
        self._engine.gather_all()
        r = self._layers.set_state_dict(sd, use_structured_name)
        self._engine.reshard_from_full()
        return r

    def get_all_parameters(self, convert2cpu=False):
        self._engine.gather_all()

    def parameters(self, include_sublayers=True):
        return self._layers.parameters(include_sublayers)

    def named_parameters(self, prefix="", include_sublayers=True, remove_duplicate=True):
        return self._layers.named_parameters(prefix, include_sublayers, remove_duplicate)


class GroupShardedOptimizer:
    def __init__(self, engine):
        self._engine = engine
        self._inner = engine.inner_opt

    def step(self):
        self._engine.step()

    def clear_grad(self, set_to_zero=True):
        self._engine.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def get_lr(self):
        return self._inner.get_lr()

    def set_lr(self, v):
        self._inner.set_lr(v)

    def state_dict(self):
        return self._inner.state_dict()

    def set_state_dict(self, sd):
        self._inner.set_state_dict(sd)

    def __getattr__(self, k):
        return getattr(self._inner, k)


def group_sharded_parallel(model, optimizer, level, scaler=None, group=None, offload=False, sync_buffers=False,
                           buffer_max_size=2 ** 23, segment_size=2 ** 20, sync_comm=False, dp_group=None,
                           exclude_layer=None):
    """level: 'os' (stage 1), 'os_g' (stage 2), 'p_g_os' (stage 3)."""
    stage = {"os": 1, "os_g": 2, "p_g_os": 3}[level]
    if not C.is_initialized() and C.get_world_size() > 1:
        C.init_parallel_env()
    mp_group = None
    from ..distributed.fleet.topology import _get_hcg
    hcg = _get_hcg()
    if hcg is not None:
        mp_group = hcg.get_model_parallel_group()
        if group is None and hcg.get_sharding_parallel_world_size() > 1:
            group = hcg.get_sharding_parallel_group()
    eng = GroupShardedEngine(model, optimizer, stage, group, mp_group=mp_group, dp_group=dp_group,
                             offload=offload)
    return GroupShardedModel(eng), GroupShardedOptimizer(eng), scaler


def save_group_sharded_model(model, output, optimizer=None):
    import os
    from ..framework.io import save
    os.makedirs(output, exist_ok=True)
    sd = model.state_dict()
    if C.get_rank() == 0:
        save(sd, os.path.join(output, "model.pdmodel"))
    if optimizer is not None:
        save(optimizer.state_dict(), os.path.join(output, f"model.pdopt.rank{C.get_rank()}"))
