"""Pipeline parallelism: LayerDesc / SharedLayerDesc / PipelineLayer and the 1F1B schedule.

Reference: python/paddle/distributed/fleet/meta_parallel/parallel_layers/pp_layers.py:57 (LayerDesc),
:258 (PipelineLayer); meta_parallel/pipeline_parallel.py:255 (PipelineParallel), :575
(forward_backward_pipeline), :820 (train_batch); pp_utils/p2p_communication.py.

Activations move between neighbouring stages with RCCL send/recv (one xGMI hop on an MI355X node);
shapes are exchanged once per micro-batch as a small int64 header so ragged last micro-batches work.
Schedule = 1F1B (warm-up = stages - stage_id - 1 forwards, then one-forward-one-backward, then
cool-down backwards), so at most `stages` micro-batch activations are alive per stage.

Interleaved 1F1B (virtual pipeline, reference pipeline_parallel.py PipelineParallelWithInterleave):
with V virtual stages each rank holds V model chunks (chunk c = v * stages + stage_id), the ring wraps
from the last stage back to the first, and the warm-up is (stages - stage_id - 1) * 2 + (V - 1) * stages
virtual micro-batches — the bubble shrinks by V. Every message carries a (kind, chunk, micro-batch)
header and each rank reads its peer's stream in send order, stashing messages it does not need yet,
so forward activations and backward gradients that share one link (always at 2 stages, and on the
ring's wrap edge) can never be mismatched, on gloo or RCCL alike.
"""
from __future__ import annotations

import re

import math

import torch
import torch.distributed as dist

from .. import nn
from ..distributed import collective as C
from ..framework.tensor import Tensor, _wrap

from .p2p import P2P  # noqa: E402

_FWD, _BWD = 0, 1


class LayerDesc:
    def __init__(self, layer_func, *inputs, **kwargs):
        self.layer_func = layer_func
        self.inputs = inputs
        self.kwargs = kwargs
        if not issubclass(layer_func, nn.Layer):
            raise TypeError("LayerDesc expects an nn.Layer subclass")

    def build_layer(self):
        return self.layer_func(*self.inputs, **self.kwargs)

    def __repr__(self):
        return f"LayerDesc({self.layer_func.__name__})"


class SharedLayerDesc(LayerDesc):
    def __init__(self, key, layer_func, forward_func=None, shared_weight_attr="weight", *inputs, **kwargs):
        super().__init__(layer_func, *inputs, **kwargs)
        self.layer_name = key
        self.forward_func = forward_func
        self.shared_weight_attr = shared_weight_attr


class _SharedCall(nn.Layer):
    def __init__(self, layer, fn):
        super().__init__()
        self.layer = layer
        self.fn = fn

    def forward(self, x):
        return self.fn(self.layer, x)


class SegmentLayers:
    """Stage boundaries of a PipelineLayer's descriptor list (reference pp_layers.py:93 SegmentLayers):

    * ``"uniform"``: equal counts, the remainder going to the LAST parts;
    * ``"layer:<regex>"``: equal numbers of the descriptors whose class / function name matches the regex
      (case-insensitive) per part — each boundary right after a part's last matching layer, so leading layers
      (embedding) join the first part and trailing ones (norm, head) the last; the count must divide evenly;
    * a list of boundaries (``[0, b1, ..]``; the final ``len(layers)`` may be left out).

    With ``num_virtual_pipeline_stage`` the list is cut into num_parts x that many chunks."""

    def __init__(self, layers_desc, num_parts, method="uniform", num_virtual_pipeline_stage=None):
        self._layers_desc = list(layers_desc)
        self.method = method
        self.num_parts = num_parts
        self.num_items = len(self._layers_desc)
        self.num_virtual_pipeline_stage = num_virtual_pipeline_stage
        self.total_parts = num_parts * (num_virtual_pipeline_stage or 1)
        if self.num_items < self.num_parts:
            raise ValueError(f"{self.num_items} layers cannot be split into {self.num_parts} pipeline stages")

    def do_segment(self):
        m = self.method
        if isinstance(m, (list, tuple)):
            b = [int(x) for x in m]
            if not b or b[0] != 0 or any(x < 0 or x > self.num_items for x in b) or b != sorted(b):
                raise ValueError(f"seg_method {list(m)}: boundaries must start at 0, ascend and stay <= "
                                 f"{self.num_items}")
            if len(b) == self.total_parts:  # last boundary left out
                b.append(self.num_items)
            if len(b) != self.total_parts + 1:
                raise ValueError(f"seg_method {list(m)} has {len(b) - 1} parts, {self.total_parts} needed")
            return b
        if m == "uniform":
            return self.uniform(self.num_items, self.total_parts)
        if isinstance(m, str) and m.startswith("layer:"):
            rx = re.compile(m.split(":", 1)[1], re.IGNORECASE)
            hits = [i for i, d in enumerate(self._layers_desc) if (nm := self._name(d)) is not None and rx.search(nm)]
            if not hits:
                raise ValueError(f"seg_method {m!r}: no layer matches")
            if len(hits) % self.total_parts:
                raise ValueError(f"seg_method {m!r}: {len(hits)} matching layers do not divide into "
                                 f"{self.total_parts} parts")
            per = len(hits) // self.total_parts
            return [0] + [hits[k * per - 1] + 1 for k in range(1, self.total_parts)] + [self.num_items]
        raise ValueError(f"seg_method {m!r} is not supported (uniform, layer:<regex> or a boundary list)")

    @staticmethod
    def _name(d):
        if isinstance(d, LayerDesc):
            f = d.layer_func
            return getattr(f, "__name__", type(f).__name__)
        if isinstance(d, nn.Layer):
            return type(d).__name__
        return getattr(d, "__name__", None)

    @staticmethod
    def uniform(num_items, num_parts):
        base, extra = divmod(num_items, num_parts)
        out = [0]
        for i in range(1, num_parts + 1):
            out.append(out[-1] + base + (1 if i > num_parts - extra else 0))
        return out


class PipelineLayer(nn.Layer):
    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seg_method="uniform",
                 recompute_interval=0, recompute_ctx=None, num_virtual_pipeline_stages=None):
        super().__init__()
        from ..distributed.fleet.topology import _get_hcg
        hcg = _get_hcg()
        if num_stages is None:
            num_stages = hcg.get_pipe_parallel_world_size() if hcg else 1
        self._num_stages = num_stages
        self._stage_id = hcg.get_stage_id() if hcg else 0
        self._loss_fn = loss_fn
        self._recompute_interval = recompute_interval
        self._layers_desc = list(layers)
        n = len(self._layers_desc)
        V = int(num_virtual_pipeline_stages or 1)
        self._num_virtual_stages = V
        self.segment_parts = self._segment(n, num_stages * V, seg_method)
        assert len(self.segment_parts) == num_stages * V + 1, self.segment_parts
        self.run_function = []
        self.shared_layers = nn.LayerDict()
        self._built = nn.LayerList()
        self._model_chunks = []
        for v in range(V):
            c = v * num_stages + self._stage_id
            lo, hi = self.segment_parts[c], self.segment_parts[c + 1]
            if v == 0:
                self._start, self._end = lo, hi
            fns = []
            for i in range(lo, hi):
                d = self._layers_desc[i]
                if isinstance(d, SharedLayerDesc):
                    if d.layer_name not in self.shared_layers:
                        self.shared_layers[d.layer_name] = d.build_layer()
                    l = self.shared_layers[d.layer_name]
                    fns.append(_SharedCall(l, d.forward_func) if d.forward_func else l)
                elif isinstance(d, LayerDesc):
                    l = d.build_layer()
                    self._built.append(l)
                    fns.append(l)
                elif isinstance(d, nn.Layer):
                    self._built.append(d)
                    fns.append(d)
                else:
                    fns.append(d)  # plain callable
            self._model_chunks.append(fns)
        self.run_function = self._model_chunks[0] if V == 1 else [f for ch in self._model_chunks for f in ch]

    def get_num_virtual_stages(self):
        return self._num_virtual_stages

    def get_model_chunks(self):
        return self._model_chunks

    def _segment(self, n, stages, method):
        return SegmentLayers(self._layers_desc, self._num_stages, method,
                             self._num_virtual_stages if self._num_virtual_stages > 1 else None).do_segment()

    def get_stage_from_index(self, idx):
        for c in range(len(self.segment_parts) - 1):
            if self.segment_parts[c] <= idx < self.segment_parts[c + 1]:
                return c % self._num_stages
        return self._num_stages - 1

    @staticmethod
    def _run(fns):
        def run(*x):
            x = x[0] if len(x) == 1 else x
            for f in fns:
                x = f(x)
            return x
        return run

    @staticmethod
    def _need_recompute(fns, inputs):
        """A segment is recomputed only if some input needs a gradient and it holds parameters."""
        if not any(isinstance(t, Tensor) and not t.stop_gradient for t in inputs):
            return False
        return any(isinstance(f, nn.Layer) and len(list(f.parameters())) > 0 for f in fns)

    def forward(self, x, chunk_id=None):
        """Run this stage's (or model chunk's) layers; with ``recompute_interval`` = k the layers go in
        consecutive segments of k, each recomputed in backward as one checkpoint (reference pp_layers.py:793)."""
        from ..distributed.fleet.recompute import recompute
        fns = self.run_function if chunk_id is None else self._model_chunks[chunk_id]
        k = self._recompute_interval
        if not k or not self.training:
            return self._run(fns)(x)
        for lo in range(0, len(fns), k):
            seg = fns[lo:lo + k]
            args = x if isinstance(x, tuple) else (x,)
            x = recompute(self._run(seg), *args) if self._need_recompute(seg, args) else self._run(seg)(*args)
        return x


class PipelineParallel(nn.Layer):
    def __init__(self, layers, hcg, strategy):
        super().__init__()
        self._layers = layers
        self._hcg = hcg
        cfg = (strategy.pipeline_configs if strategy is not None else {}) or {}
        self.accumulate_steps = int(cfg.get("accumulate_steps", 1))
        self.micro_batch_size = int(cfg.get("micro_batch_size", 1))
        self.num_stages = hcg.get_pipe_parallel_world_size()
        self.stage_id = hcg.get_stage_id()
        self.group = hcg.get_pipe_parallel_group()
        self.is_first = self.stage_id == 0
        self.is_last = self.stage_id == self.num_stages - 1
        self.prev_rank = self.group.ranks[self.stage_id - 1] if not self.is_first else None
        self.next_rank = self.group.ranks[self.stage_id + 1] if not self.is_last else None
        self._dp_sync = hcg.get_data_parallel_world_size() > 1
        self._p2p = None
        self._p2p_ordered = True  # 1F1B / FThenB / ZBH1 consume each directed channel in production order
        # job order of the non-interleaved schedule (parallel/pp_schedules.py; ZBH1 is its own class)
        mode = str(cfg.get("schedule_mode", "1F1B")).upper()
        self.schedule_mode = mode if mode in ("1F1B", "FTHENB", "EAGER1F1B") else "1F1B"

    # --------------------------------------------------------------- p2p
    def _dev(self):
        p = next(iter(self._layers.parameters()), None)
        return p._t.device if p is not None else torch.device("cpu")

    def _p2p_chan(self):
        """The stage's tagged p2p endpoint (parallel/p2p.py: tags + meta on the host twin of the pipe group, meta
        once per shape, payloads on the pipe group's RCCL communicator)."""
        if self._p2p is None:
            host = self._hcg.get_pipe_parallel_host_group() if hasattr(self._hcg, "get_pipe_parallel_host_group") \
                else None
            down = self._hcg.get_pipe_parallel_down_group() if hasattr(self._hcg, "get_pipe_parallel_down_group") \
                else None
            # ordered (no per-message header) unless the schedule consumes a channel out of production order
            self._p2p = P2P(self._dev(), self.group.process_group, host, ordered=self._p2p_ordered,
                            record=getattr(self, "_p2p_record", False), down_group=down)
        return self._p2p

    def _send(self, t, dst, kind=_FWD, key=(0, 0)):
        # non-blocking: a stage may send its next activation before the neighbour has posted the
        # receive (1F1B would dead-lock on rendezvous sends); buffers are kept alive until joined
        self._p2p_chan().send(t, dst, (kind, key[0], key[1]))

    def _join_sends(self):
        if self._p2p is not None:
            self._p2p.join()

    def _recv(self, src, kind=_FWD, key=(0, 0)):
        """The (kind, key) message from ``src`` (messages that arrive ahead of it are stashed)."""
        return self._p2p_chan().recv(src, (kind, key[0], key[1]))

    # --------------------------------------------------------------- schedule
    def _split(self, data):
        if isinstance(data, (list, tuple)):
            parts = [self._split(d) for d in data]
            return list(zip(*parts))
        t = data._t if isinstance(data, Tensor) else data
        n = self.accumulate_steps
        return [_wrap(c) for c in t.chunk(n, 0)]

    def _flush(self):
        """A job that receives nothing issues the sends the previous job queued before its compute (p2p.py)."""
        if self._p2p is not None:
            self._p2p.flush()

    def _forward_step(self, mb_input, mb_label, mb=0):
        if self.is_first:
            self._flush()
            x = mb_input
        else:
            xt = self._recv(self.prev_rank, _FWD, (0, mb)).requires_grad_(True)
            x = _wrap(xt)
        out = self._layers(x)
        if self.is_last:
            loss = self._layers._loss_fn(out, mb_label) if self._layers._loss_fn is not None else out
            return x, loss
        self._send(out._t.detach(), self.next_rank, _FWD, (0, mb))
        return x, out

    def _backward_step(self, inp, out, mb=0):
        if self.is_last:
            self._flush()
            (out._t / self.accumulate_steps).backward()
        else:
            g = self._recv(self.next_rank, _BWD, (0, mb))
            out._t.backward(g)
        if not self.is_first:
            self._send(inp._t.grad, self.prev_rank, _BWD, (0, mb))

    def forward_backward_pipeline(self, data, scaler=None):
        self._p2p_chan().begin_run()
        inputs, labels = (data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None))
        mb_in = self._split(inputs) if self.is_first else [None] * self.accumulate_steps
        mb_lb = self._split(labels) if (self.is_last and labels is not None) else [None] * self.accumulate_steps
        from .pp_schedules import schedule
        queue, losses = {}, []
        # 1F1B (default), FThenB or Eager1F1B job list of this stage: F = forward of micro-batch mb (its input
        # received from the previous stage), B = its backward (the output gradient received from the next stage)
        self.jobs = schedule(self.schedule_mode, self.num_stages, self.stage_id, self.accumulate_steps)
        for kind, mb in self.jobs:
            if kind == "F":
                x, y = self._forward_step(mb_in[mb], mb_lb[mb], mb)
                queue[mb] = (x, y)
                if self.is_last:
                    losses.append(y)
            else:
                inp, out = queue.pop(mb)
                self._backward_step(inp, out, mb)
        return self._finish(losses)

    def _finish(self, losses):
        self._join_sends()
        if self._dp_sync:
            # PP x DP: the stage's gradients averaged over its data-parallel group in flat per-dtype buckets (reference
            # hybrid_parallel_util.fused_allreduce_gradients), not one all-reduce + scale per parameter
            from ..distributed.fleet.utils.hybrid_parallel_util import fused_allreduce_gradients
            fused_allreduce_gradients(list(self._layers.parameters()), self._hcg)
        # broadcast the mean loss from the last stage
        loss = torch.zeros((), device=self._dev())
        if self.is_last and losses:
            loss = torch.stack([l._t.detach().float() for l in losses]).mean()
        if self.num_stages > 1:
            dist.broadcast(loss, self.group.ranks[-1], group=self.group.process_group)
        return _wrap(loss)

    def _fuse_grad_accumulation(self):
        from ..ops.linear import fuse_grad_accumulation
        self._mg_params = fuse_grad_accumulation(self._layers, getattr(self, "_mg_params", None))

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None):
        self._layers.train()
        self._fuse_grad_accumulation()
        loss = self.forward_backward_pipeline(data, scaler)
        optimizer.step()
        optimizer.clear_grad()
        if lr_scheduler is not None:
            lr_scheduler.step()
        from ..distributed import collective_check as _cc
        if _cc.enabled():
            _cc.check_collectives("pipeline train_batch")
        return loss

    @torch.no_grad()
    def eval_batch(self, data, compute_loss=True):
        self._layers.eval()
        self._p2p_chan().begin_run()
        inputs, labels = (data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None))
        mb_in = self._split(inputs) if self.is_first else [None] * self.accumulate_steps
        mb_lb = self._split(labels) if (self.is_last and labels is not None) else [None] * self.accumulate_steps
        outs = []
        for i in range(self.accumulate_steps):
            _, y = self._forward_step(mb_in[i], mb_lb[i] if compute_loss else None, i)
            if self.is_last:
                outs.append(y._t.float().mean() if compute_loss else y._t)
        self._join_sends()
        if self.is_last and compute_loss:
            return _wrap(torch.stack(outs).mean())
        return outs

    def forward(self, *a, **k):
        return self._layers(*a, **k)

    def parameters(self, include_sublayers=True):
        return self._layers.parameters(include_sublayers)


class PipelineParallelZeroBubble(PipelineParallel):
    """1F1B with the backward split into input-gradient (B) and deferred weight-gradient (W) jobs — the
    reference's ZBH1 schedule (distributed/passes/pipeline_scheduler_pass/pipeline_zero_bubble.py:61), picked
    by fleet for ``pipeline_configs["schedule_mode"] = "ZBH1"``. Job order: parallel/pp_schedules.py zbh1;
    the W jobs run the linears' dW GEMMs recorded during B (ops/linear.py defer_weight_grads)."""

    def forward_backward_pipeline(self, data, scaler=None):
        from ..ops import linear as LIN
        from .pp_schedules import zbh1
        self._p2p_chan().begin_run()
        inputs, labels = (data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None))
        n = self.accumulate_steps
        mb_in = self._split(inputs) if self.is_first else [None] * n
        mb_lb = self._split(labels) if (self.is_last and labels is not None) else [None] * n
        store, wq, losses = {}, {}, []
        self.jobs = zbh1(self.num_stages, self.stage_id, n)
        self.deferred_wgrads = 0
        for kind, mb in self.jobs:
            if kind == "F":
                with LIN.zero_bubble_forward():
                    x, y = self._forward_step(mb_in[mb], mb_lb[mb], mb)
                store[mb] = (x, y)
                if self.is_last:
                    losses.append(y)
            elif kind == "B":
                q = []
                with LIN.defer_weight_grads(q):
                    self._backward_step(*store.pop(mb), mb)
                wq[mb] = q
                self.deferred_wgrads += len(q)
            else:
                self._flush()
                LIN.apply_weight_grads(wq.pop(mb))
        return self._finish(losses)




class PipelineParallelWithInterleave(PipelineParallel):
    """Interleaved 1F1B over V model chunks per rank (reference:
    fleet/meta_parallel/pipeline_parallel.py PipelineParallelWithInterleave). accumulate_steps must be a
    multiple of the number of stages; chunk v of stage s computes layers segment v * stages + s."""

    def __init__(self, layers, hcg, strategy):
        super().__init__(layers, hcg, strategy)
        self.V = layers.get_num_virtual_stages()
        if self.V < 2:
            raise ValueError("PipelineParallelWithInterleave needs num_virtual_pipeline_stages >= 2")
        S = self.num_stages
        self.prev_rank = self.group.ranks[(self.stage_id - 1) % S]
        self.next_rank = self.group.ranks[(self.stage_id + 1) % S]
        self._p2p_ordered = False  # chunks of a ring channel are consumed out of production order: tagged + stash
        if self.accumulate_steps % S:
            raise ValueError(f"accumulate_steps ({self.accumulate_steps}) must be a multiple of the "
                             f"pipeline degree ({S}) for the interleaved schedule")

    def _chunk_of(self, k, forward):
        from .pp_schedules import vpp_chunk
        return vpp_chunk(k, self.num_stages, self.V, forward)

    def _mb_of(self, k):
        from .pp_schedules import vpp_mb
        return vpp_mb(k, self.num_stages, self.V)

    def _vforward(self, k, mb_in, mb_lb, store, losses):
        v, mb = self._chunk_of(k, True), self._mb_of(k)
        first = self.stage_id == 0 and v == 0
        last = self.stage_id == self.num_stages - 1 and v == self.V - 1
        if first:
            self._flush()
            x = mb_in[mb]
        else:
            # chunk v of stage 0 consumes chunk v-1 of the last stage (ring wrap)
            x = _wrap(self._recv(self.prev_rank, _FWD, (v if self.stage_id else v - 1, mb)).requires_grad_(True))
        out = self._layers(x, chunk_id=v)
        if last:
            out = self._layers._loss_fn(out, mb_lb[mb]) if self._layers._loss_fn is not None else out
            losses.append(out)
        else:
            self._send(out._t.detach(), self.next_rank, _FWD, (v, mb))
        store[(v, mb)] = (x, out)

    def _vbackward(self, k, store):
        v, mb = self._chunk_of(k, False), self._mb_of(k)
        first = self.stage_id == 0 and v == 0
        last = self.stage_id == self.num_stages - 1 and v == self.V - 1
        x, out = store.pop((v, mb))
        if last:
            self._flush()
            (out._t / self.accumulate_steps).backward()
        else:
            # the gradient of chunk v's output comes from chunk v (or v+1 across the wrap) downstream
            src_v = v + 1 if self.stage_id == self.num_stages - 1 else v
            out._t.backward(self._recv(self.next_rank, _BWD, (src_v, mb)))
        if not first:
            self._send(x._t.grad, self.prev_rank, _BWD, (v, mb))

    def forward_backward_pipeline(self, data, scaler=None):
        inputs, labels = (data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None))
        n = self.accumulate_steps
        mb_in = self._split(inputs) if self.stage_id == 0 else [None] * n
        mb_lb = self._split(labels) if (self.stage_id == self.num_stages - 1 and labels is not None) else [None] * n
        from .pp_schedules import vpp
        store, losses = {}, []
        self.jobs = vpp(self.num_stages, self.stage_id, n, self.V)  # interleaved 1F1B job list of this stage
        for kind, k in self.jobs:
            if kind == "F":
                self._vforward(k, mb_in, mb_lb, store, losses)
            else:
                self._vbackward(k, store)
        self.is_last = self.stage_id == self.num_stages - 1  # loss lives on the last stage's last chunk
        return self._finish(losses)

    @torch.no_grad()
    def eval_batch(self, data, compute_loss=True):
        self._layers.eval()
        inputs, labels = (data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None))
        n = self.accumulate_steps
        mb_in = self._split(inputs) if self.stage_id == 0 else [None] * n
        mb_lb = self._split(labels) if (self.stage_id == self.num_stages - 1 and labels is not None) else [None] * n
        store, losses = {}, []
        for k in range(n * self.V):
            self._vforward(k, mb_in, mb_lb if compute_loss else [None] * n, store, losses)
        self._join_sends()
        if self.stage_id == self.num_stages - 1 and compute_loss:
            return _wrap(torch.stack([l._t.float().mean() for l in losses]).mean())
        return [l._t for l in losses]


class PipelineParallelZeroBubbleVPP(PipelineParallelWithInterleave):
    """Interleaved pipeline with the weight gradients split off (reference ZBVPP,
    distributed/passes/pipeline_scheduler_pass/pipeline_zero_bubble.py; fleet picks it for
    ``schedule_mode = "ZBVPP"`` with virtual stages): job order parallel/pp_schedules.py zbvpp; a B job runs the
    chunk's input gradient with the linears' dW GEMMs recorded (ops/linear.py defer_weight_grads), its W job runs
    them later — in the cool-down, while the stage would otherwise wait for the next gradient from downstream."""

    def forward_backward_pipeline(self, data, scaler=None):
        from ..ops import linear as LIN
        from .pp_schedules import zbvpp
        inputs, labels = (data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None))
        n = self.accumulate_steps
        mb_in = self._split(inputs) if self.stage_id == 0 else [None] * n
        mb_lb = self._split(labels) if (self.stage_id == self.num_stages - 1 and labels is not None) else [None] * n
        store, wq, losses = {}, {}, []
        self.jobs = zbvpp(self.num_stages, self.stage_id, n, self.V)
        self.deferred_wgrads = 0
        for kind, k in self.jobs:
            if kind == "F":
                with LIN.zero_bubble_forward():
                    self._vforward(k, mb_in, mb_lb, store, losses)
            elif kind == "B":
                q = []
                with LIN.defer_weight_grads(q):
                    self._vbackward(k, store)
                wq[k] = q
                self.deferred_wgrads += len(q)
            else:
                self._flush()
                LIN.apply_weight_grads(wq.pop(k))
        self.is_last = self.stage_id == self.num_stages - 1
        return self._finish(losses)


class PipelineParallelWithInterleaveFthenB(PipelineParallelWithInterleave):
    """Virtual pipeline that runs every forward micro-step first, then every backward (reference
    pipeline_parallel.py:2261 PipelineParallelWithInterleaveFthenB, chosen by fleet when
    pp <= accumulate_steps < 2 * pp). Micro-step k runs chunk (k // accumulate_steps) on micro-batch
    k % accumulate_steps; backward walks the chunks in reverse. Messages are keyed by (chunk, micro-batch),
    so the all-forward order needs no extra synchronisation."""

    def __init__(self, layers, hcg, strategy):
        PipelineParallel.__init__(self, layers, hcg, strategy)
        self.V = layers.get_num_virtual_stages()
        if self.V < 2:
            raise ValueError("PipelineParallelWithInterleaveFthenB needs num_virtual_pipeline_stages >= 2")
        S = self.num_stages
        self.prev_rank = self.group.ranks[(self.stage_id - 1) % S]
        self.next_rank = self.group.ranks[(self.stage_id + 1) % S]
        self._p2p_ordered = False  # chunks of a ring channel are consumed out of production order: tagged + stash
        if self.accumulate_steps < S:
            raise ValueError(f"accumulate_steps ({self.accumulate_steps}) must be >= pp degree ({S})")

    def _chunk_of(self, k, forward):
        v = (k // self.accumulate_steps) % self.V
        return v if forward else self.V - 1 - v

    def _mb_of(self, k):
        return k % self.accumulate_steps

    def forward_backward_pipeline(self, data, scaler=None):
        inputs, labels = (data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None))
        n = self.accumulate_steps
        mb_in = self._split(inputs) if self.stage_id == 0 else [None] * n
        mb_lb = self._split(labels) if (self.stage_id == self.num_stages - 1 and labels is not None) else [None] * n
        store, losses = {}, []
        for k in range(n * self.V):
            self._vforward(k, mb_in, mb_lb, store, losses)
        for k in range(n * self.V):
            self._vbackward(k, store)
        self.is_last = self.stage_id == self.num_stages - 1
        return self._finish(losses)
