"""Pipeline parallelism: LayerDesc / SharedLayerDesc / PipelineLayer and the 1F1B schedule.

Reference: python/paddle/distributed/fleet/meta_parallel/parallel_layers/pp_layers.py:57 (LayerDesc),
:258 (PipelineLayer); meta_parallel/pipeline_parallel.py:255 (PipelineParallel), :575
(forward_backward_pipeline), :820 (train_batch); pp_utils/p2p_communication.py.

Activations move between neighbouring stages with RCCL send/recv (one xGMI hop on an MI355X node);
shapes are exchanged once per micro-batch as a small int64 header so ragged last micro-batches work.
Schedule = 1F1B (warm-up = stages - stage_id - 1 forwards, then one-forward-one-backward, then
cool-down backwards), so at most `stages` micro-batch activations are alive per stage.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from .. import nn
from ..distributed import collective as C
from ..framework.tensor import Tensor, _wrap


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
        self.segment_parts = self._segment(n, num_stages, seg_method)
        lo, hi = self.segment_parts[self._stage_id], self.segment_parts[self._stage_id + 1]
        self._start, self._end = lo, hi
        self.run_function = []
        self.shared_layers = nn.LayerDict()
        self._built = nn.LayerList()
        for i in range(lo, hi):
            d = self._layers_desc[i]
            if isinstance(d, SharedLayerDesc):
                if d.layer_name not in self.shared_layers:
                    self.shared_layers[d.layer_name] = d.build_layer()
                l = self.shared_layers[d.layer_name]
                self.run_function.append(_SharedCall(l, d.forward_func) if d.forward_func else l)
            elif isinstance(d, LayerDesc):
                l = d.build_layer()
                self._built.append(l)
                self.run_function.append(l)
            elif isinstance(d, nn.Layer):
                self._built.append(d)
                self.run_function.append(d)
            else:
                self.run_function.append(d)  # plain callable

    @staticmethod
    def _segment(n, stages, method):
        if isinstance(method, (list, tuple)):
            return list(method)
        base = n // stages
        extra = n % stages
        parts = [0]
        for s in range(stages):
            parts.append(parts[-1] + base + (1 if s < extra else 0))
        return parts

    def get_stage_from_index(self, idx):
        for s in range(self._num_stages):
            if self.segment_parts[s] <= idx < self.segment_parts[s + 1]:
                return s
        return self._num_stages - 1

    def forward(self, x):
        from ..distributed.fleet.recompute import recompute
        for i, f in enumerate(self.run_function):
            if self._recompute_interval and self.training and i % self._recompute_interval == 0 and \
                    isinstance(f, nn.Layer):
                x = recompute(f, x)
            else:
                x = f(x)
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
        self._pending = []

    # --------------------------------------------------------------- p2p
    def _dev(self):
        p = next(iter(self._layers.parameters()), None)
        return p._t.device if p is not None else torch.device("cpu")

    def _send(self, t, dst):
        # non-blocking: a stage may send its next activation before the neighbour has posted the
        # receive (1F1B would dead-lock on rendezvous sends); buffers are kept alive until joined
        t = t.contiguous()
        hdr = torch.tensor([t.dim()] + list(t.shape) + [0] * (8 - t.dim()) + [_DT_CODE[t.dtype]], dtype=torch.int64,
                           device=t.device)
        pg = self.group.process_group
        self._pending.append((dist.isend(hdr, dst, group=pg), hdr))
        self._pending.append((dist.isend(t, dst, group=pg), t))

    def _join_sends(self):
        for w, _ in self._pending:
            w.wait()
        self._pending = []

    def _recv(self, src):
        hdr = torch.empty(10, dtype=torch.int64, device=self._dev())
        dist.recv(hdr, src, group=self.group.process_group)
        nd = int(hdr[0])
        shape = [int(v) for v in hdr[1:1 + nd]]
        t = torch.empty(shape, dtype=_CODE_DT[int(hdr[9])], device=self._dev())
        dist.recv(t, src, group=self.group.process_group)
        return t

    # --------------------------------------------------------------- schedule
    def _split(self, data):
        if isinstance(data, (list, tuple)):
            parts = [self._split(d) for d in data]
            return list(zip(*parts))
        t = data._t if isinstance(data, Tensor) else data
        n = self.accumulate_steps
        return [_wrap(c) for c in t.chunk(n, 0)]

    def _forward_step(self, mb_input, mb_label):
        if self.is_first:
            x = mb_input
        else:
            xt = self._recv(self.prev_rank).requires_grad_(True)
            x = _wrap(xt)
        out = self._layers(x)
        if self.is_last:
            loss = self._layers._loss_fn(out, mb_label) if self._layers._loss_fn is not None else out
            return x, loss
        self._send(out._t.detach(), self.next_rank)
        return x, out

    def _backward_step(self, inp, out):
        if self.is_last:
            (out._t / self.accumulate_steps).backward()
        else:
            g = self._recv(self.next_rank)
            out._t.backward(g)
        if not self.is_first:
            self._send(inp._t.grad, self.prev_rank)

    def forward_backward_pipeline(self, data, scaler=None):
        inputs, labels = (data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None))
        mb_in = self._split(inputs) if self.is_first else [None] * self.accumulate_steps
        mb_lb = self._split(labels) if (self.is_last and labels is not None) else [None] * self.accumulate_steps
        n = self.accumulate_steps
        warm = min(self.num_stages - self.stage_id - 1, n)
        steady = n - warm
        queue = []
        losses = []
        fi = 0
        for _ in range(warm):
            x, y = self._forward_step(mb_in[fi], mb_lb[fi])
            queue.append((x, y))
            if self.is_last:
                losses.append(y)
            fi += 1
        for i in range(steady):
            x, y = self._forward_step(mb_in[fi], mb_lb[fi])
            queue.append((x, y))
            if self.is_last:
                losses.append(y)
            fi += 1
            inp, out = queue.pop(0)
            self._backward_step(inp, out)
        for _ in range(warm):
            inp, out = queue.pop(0)
            self._backward_step(inp, out)
        self._join_sends()
        if self._dp_sync:
            g = self._hcg.get_data_parallel_group()
            for p in self._layers.parameters():
                if p._t.grad is not None:
                    dist.all_reduce(p._t.grad, op=dist.ReduceOp.SUM, group=g.process_group)
                    p._t.grad.mul_(1.0 / g.nranks)
        # broadcast the mean loss from the last stage
        loss = torch.zeros((), device=self._dev())
        if self.is_last and losses:
            loss = torch.stack([l._t.detach().float() for l in losses]).mean()
        if self.num_stages > 1:
            dist.broadcast(loss, self.group.ranks[-1], group=self.group.process_group)
        return _wrap(loss)

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None):
        self._layers.train()
        loss = self.forward_backward_pipeline(data, scaler)
        optimizer.step()
        optimizer.clear_grad()
        if lr_scheduler is not None:
            lr_scheduler.step()
        return loss

    @torch.no_grad()
    def eval_batch(self, data, compute_loss=True):
        self._layers.eval()
        inputs, labels = (data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None))
        mb_in = self._split(inputs) if self.is_first else [None] * self.accumulate_steps
        mb_lb = self._split(labels) if (self.is_last and labels is not None) else [None] * self.accumulate_steps
        outs = []
        for i in range(self.accumulate_steps):
            _, y = self._forward_step(mb_in[i], mb_lb[i] if compute_loss else None)
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


_DT_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.int64: 3, torch.int32: 4, torch.bool: 5}
_CODE_DT = {v: k for k, v in _DT_CODE.items()}
