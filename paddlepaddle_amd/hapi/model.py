"""hapi high-level Model API. Reference: python/paddle/hapi/model.py (Model: prepare/fit/evaluate/
predict/train_batch/eval_batch/predict_batch/save/load/summary; DynamicGraphAdapter).

One process per GPU: under ``paddle.distributed`` (world_size > 1) the network is wrapped in our
bucketed RCCL DataParallel and datasets are split with DistributedBatchSampler; eval metrics are
all-gathered before accumulation.
"""
from __future__ import annotations

import inspect
import os
import time

import numpy as np
import torch

from ..framework.tensor import Tensor, _wrap
from ..framework import io as _io
from ..io import DataLoader, Dataset, DistributedBatchSampler
from ..metric import Metric
from . import callbacks as cbks_mod


def _to_list(x):
    if x is None:
        return []
    return list(x) if isinstance(x, (list, tuple)) else [x]


def _to_tensor(x):
    if isinstance(x, Tensor):
        return x
    from ..framework.tensor import to_tensor
    return to_tensor(np.asarray(x))


def _np(x):
    return x.numpy() if isinstance(x, Tensor) else np.asarray(x)


class Model:
    def __init__(self, network, inputs=None, labels=None):
        self.network = network
        self._inputs = _to_list(inputs)
        self._labels = _to_list(labels)
        self._optimizer = None
        self._loss = None
        self._metrics = []
        self._amp_level = "O0"
        self._scaler = None
        self._amp_dtype = "float16"
        self.stop_training = False
        self.mode = "train"
        self._save_dir = None
        self._accumulate = 1
        self._dp = None
        self._n_inputs = len(self._inputs) if self._inputs else self._forward_arity()
        from ..distributed import collective as C
        self._world = C.get_world_size() if C.is_initialized() else 1

    def _forward_arity(self):
        try:
            sig = inspect.signature(self.network.forward)
            return max(1, sum(1 for p in sig.parameters.values()
                              if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD) and p.default is p.empty))
        except (TypeError, ValueError):
            return 1

    # ------------------------------------------------------------------ setup
    def prepare(self, optimizer=None, loss=None, metrics=None, amp_configs=None):
        self._optimizer = optimizer
        self._loss = loss
        self._metrics = _to_list(metrics)
        for m in self._metrics:
            if not isinstance(m, Metric):
                raise TypeError(f"{m} is not a paddle.metric.Metric")
        if amp_configs is not None:
            if isinstance(amp_configs, str):
                amp_configs = {"level": amp_configs}
            self._amp_level = amp_configs.get("level", "O1")
            self._amp_dtype = amp_configs.get("dtype", "float16")
            if self._amp_level != "O0" and self._amp_dtype == "float16":
                from ..amp import GradScaler
                self._scaler = GradScaler(init_loss_scaling=amp_configs.get("init_loss_scaling", 2.0 ** 15))
            if self._amp_level == "O2":
                from ..amp import decorate
                self.network, self._optimizer = decorate(self.network, self._optimizer, level="O2",
                                                         dtype=self._amp_dtype)
        if self._world > 1 and self._dp is None:
            from ..parallel.data_parallel import DataParallel
            self._dp = DataParallel(self.network)

    def parameters(self, *args, **kwargs):
        return self.network.parameters(*args, **kwargs)

    def _net(self):
        return self._dp if self._dp is not None else self.network

    def _autocast(self):
        if self._amp_level == "O0":
            import contextlib
            return contextlib.nullcontext()
        from ..amp import auto_cast
        return auto_cast(True, level=self._amp_level, dtype=self._amp_dtype)

    # ------------------------------------------------------------------ batches
    def _split(self, data):
        data = _to_list(data)
        n = self._n_inputs if len(data) > self._n_inputs else len(data)
        return [_to_tensor(d) for d in data[:n]], [_to_tensor(d) for d in data[n:]]

    def _compute_loss(self, outs, labels):
        if self._loss is None:
            return None
        loss = self._loss(*(_to_list(outs) + labels))
        if isinstance(loss, (list, tuple)):
            loss = sum(loss[1:], loss[0])
        return loss

    def _metric_update(self, outs, labels):
        res = []
        for m in self._metrics:
            r = m.compute(*(_to_list(outs) + labels))
            r = _to_list(r)
            if self._world > 1:
                from .. import distributed as dist
                g = []
                for t in r:
                    lst = []
                    dist.all_gather(lst, t)
                    g.append(_wrap(torch.cat([x._t for x in lst], 0)))
                r = g
            res.append(m.update(*[_np(x) for x in r]))
        return res

    def train_batch(self, inputs, labels=None, update=True):
        self.network.train()
        self.mode = "train"
        inputs = [_to_tensor(x) for x in _to_list(inputs)]
        labels = [_to_tensor(x) for x in _to_list(labels)]
        with self._autocast():
            outs = self._net()(*inputs)
            loss = self._compute_loss(outs, labels)
        scaled = loss / self._accumulate if self._accumulate > 1 else loss
        if self._scaler is not None:
            self._scaler.scale(scaled).backward()
        else:
            scaled.backward()
        if update:
            if self._scaler is not None:
                self._scaler.step(self._optimizer)
                self._scaler.update()
            else:
                self._optimizer.step()
            self._optimizer.clear_grad()
        metrics = self._metric_update(outs, labels)
        lv = [float(loss)]
        return (lv, metrics) if self._metrics else lv

    def eval_batch(self, inputs, labels=None):
        self.network.eval()
        self.mode = "eval"
        from ..framework.grad_mode import no_grad
        inputs = [_to_tensor(x) for x in _to_list(inputs)]
        labels = [_to_tensor(x) for x in _to_list(labels)]
        with no_grad(), self._autocast():
            outs = self.network(*inputs)
            loss = self._compute_loss(outs, labels) if labels else None
        metrics = self._metric_update(outs, labels)
        lv = [float(loss)] if loss is not None else []
        return (lv, metrics) if self._metrics else lv

    def predict_batch(self, inputs):
        self.network.eval()
        self.mode = "test"
        from ..framework.grad_mode import no_grad
        inputs = [_to_tensor(x) for x in _to_list(inputs)]
        with no_grad(), self._autocast():
            outs = self.network(*inputs)
        return [_np(o) for o in _to_list(outs)]

    # ------------------------------------------------------------------ loops
    def _loader(self, data, batch_size, shuffle, drop_last, num_workers):
        if data is None or isinstance(data, DataLoader):
            return data
        if isinstance(data, Dataset) or hasattr(data, "__getitem__"):
            if self._world > 1:
                bs = DistributedBatchSampler(data, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last)
                return DataLoader(data, batch_sampler=bs, num_workers=num_workers)
            return DataLoader(data, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last,
                              num_workers=num_workers)
        return data  # any iterable of batches

    def _logs(self, losses, metrics_res, step, bs):
        logs = {}
        if losses:
            logs["loss"] = losses
        for m, r in zip(self._metrics, metrics_res):
            names = _to_list(m.name())
            vals = _to_list(r)
            for n, v in zip(names, vals):
                logs[n] = v
        logs["step"] = step
        logs["batch_size"] = bs
        return logs

    def fit(self, train_data=None, eval_data=None, batch_size=1, epochs=1, eval_freq=1, log_freq=10, save_dir=None,
            save_freq=1, verbose=2, drop_last=False, shuffle=True, num_workers=0, callbacks=None,
            accumulate_grad_batches=1, num_iters=None):
        assert train_data is not None, "train_data must be given"
        self._accumulate = max(1, int(accumulate_grad_batches))
        self._save_dir = save_dir
        loader = self._loader(train_data, batch_size, shuffle, drop_last, num_workers)
        eval_loader = self._loader(eval_data, batch_size, False, False, num_workers)
        steps = len(loader) if hasattr(loader, "__len__") else None
        cb = cbks_mod.config_callbacks(callbacks, model=self, batch_size=batch_size, epochs=epochs, steps=steps,
                                       log_freq=log_freq, verbose=verbose, save_freq=save_freq,
                                       save_dir=save_dir if (self._world == 1 or _rank0()) else None,
                                       metrics=["loss"] + [n for m in self._metrics for n in _to_list(m.name())])
        self.stop_training = False
        cb.on_train_begin()
        it = 0
        for epoch in range(epochs):
            for m in self._metrics:
                m.reset()
            cb.on_epoch_begin(epoch)
            logs = {}
            for step, data in enumerate(loader):
                cb.on_train_batch_begin(step)
                ins, lbs = self._split(data)
                update = (step + 1) % self._accumulate == 0 or (steps is not None and step + 1 == steps)
                res = self.train_batch(ins, lbs, update=update)
                losses, mres = (res if self._metrics else (res, []))
                logs = self._logs(losses, mres, step, ins[0].shape[0] if ins else batch_size)
                cb.on_train_batch_end(step, logs)
                it += 1
                if num_iters is not None and it >= num_iters:
                    self.stop_training = True
                    break
            if self._metrics:
                for m in self._metrics:
                    for n, v in zip(_to_list(m.name()), _to_list(m.accumulate())):
                        logs[n] = v
            cb.on_epoch_end(epoch, logs)
            if eval_loader is not None and (epoch + 1) % eval_freq == 0:
                self._run_eval(eval_loader, cb, log_freq)
            if self.stop_training:
                break
        cb.on_train_end(logs)

    def _run_eval(self, loader, cb, log_freq=10, num_iters=None):
        for m in self._metrics:
            m.reset()
        cb.on_eval_begin({"steps": len(loader) if hasattr(loader, "__len__") else None})
        tot_loss, n, samples = 0.0, 0, 0
        for step, data in enumerate(loader):
            cb.on_eval_batch_begin(step)
            ins, lbs = self._split(data)
            res = self.eval_batch(ins, lbs)
            losses = res[0] if self._metrics else res
            if losses:
                tot_loss += losses[0]
                n += 1
            samples += ins[0].shape[0] if ins else 0
            cb.on_eval_batch_end(step, {"loss": losses})
            if num_iters is not None and step + 1 >= num_iters:
                break
        logs = {}
        if n:
            logs["loss"] = [tot_loss / n]
        for m in self._metrics:
            for name, v in zip(_to_list(m.name()), _to_list(m.accumulate())):
                logs[name] = v
        logs["samples"] = samples
        cb.on_eval_end(logs)
        return logs

    def evaluate(self, eval_data, batch_size=1, log_freq=10, verbose=2, num_workers=0, callbacks=None,
                 num_iters=None):
        loader = self._loader(eval_data, batch_size, False, False, num_workers)
        cb = cbks_mod.config_callbacks(callbacks, model=self, batch_size=batch_size, log_freq=log_freq,
                                       verbose=verbose, mode="eval")
        logs = self._run_eval(loader, cb, log_freq, num_iters)
        logs.pop("samples", None)
        return logs

    def predict(self, test_data, batch_size=1, num_workers=0, stack_outputs=False, verbose=1, callbacks=None):
        loader = self._loader(test_data, batch_size, False, False, num_workers)
        outputs = None
        for data in loader:
            data = _to_list(data)
            ins = data[:self._n_inputs] if len(data) > self._n_inputs else data
            outs = self.predict_batch(ins)
            if outputs is None:
                outputs = [[] for _ in outs]
            for i, o in enumerate(outs):
                outputs[i].append(o)
        outputs = outputs or []
        if stack_outputs:
            outputs = [np.concatenate(o, 0) for o in outputs]
        return outputs

    # ------------------------------------------------------------------ io
    def save(self, path, training=True):
        if not _rank0():
            return
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if training:
            _io.save(self.network.state_dict(), path + ".pdparams")
            if self._optimizer is not None:
                _io.save(self._optimizer.state_dict(), path + ".pdopt")
        else:
            from ..jit import save as jit_save
            specs = self._inputs or None
            jit_save(self.network, path, input_spec=specs)

    def load(self, path, skip_mismatch=False, reset_optimizer=False):
        sd = _io.load(path + ".pdparams" if not path.endswith(".pdparams") else path)
        if skip_mismatch:
            own = self.network.state_dict()
            sd = {k: v for k, v in sd.items() if k in own and list(own[k].shape) == list(v.shape)}
        self.network.set_state_dict(sd)
        opt_path = (path[:-len(".pdparams")] if path.endswith(".pdparams") else path) + ".pdopt"
        if not reset_optimizer and self._optimizer is not None and os.path.exists(opt_path):
            self._optimizer.set_state_dict(_io.load(opt_path))

    def summary(self, input_size=None, dtype=None):
        from .model_summary import summary
        if input_size is None and self._inputs:
            input_size = [tuple(s.shape) for s in self._inputs]
        return summary(self.network, input_size, dtype)


def _rank0():
    from ..distributed import collective as C
    return (not C.is_initialized()) or C.get_rank() == 0
