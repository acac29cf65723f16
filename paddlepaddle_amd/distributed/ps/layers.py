"""Trainer-side layers of parameter-server training.

Reference: python/paddle/static/nn/common.py sparse_embedding (a lookup into a server-side
MemorySparseTable, with entry admission and slot / show-click statistics) and the PS optimizer pass
(python/paddle/distributed/ps/utils/public.py / fleet/meta_optimizers/ps_optimizer.py: dense parameters
are updated on the servers, sparse tables by the pushes of the lookup's backward).
"""
from __future__ import annotations

import torch

from ...framework.tensor import Tensor, _wrap
from ...nn.layer.layers import Layer
from . import the_one_ps as _ps

_RULE_OF = {"SGD": "sgd", "Momentum": "sgd", "Adagrad": "adagrad", "Adam": "adam", "AdamW": "adam",
            "Lamb": "adam"}


def _entry_cfg(entry):
    if entry is None:
        return (0, 0.0)
    name = getattr(entry, "_name", "")
    if name == "count_filter_entry":
        return (1, float(entry._args[0]))
    if name == "probability_entry":
        return (2, float(entry._args[0]))
    return (0, 0.0)  # show_click_entry: statistics come from the show / click inputs


class DistributedEmbedding(Layer):
    """Embedding whose table lives on the parameter servers: ``size = [vocab (unused / unbounded), dim]``.
    Forward pulls the rows of the batch's unique ids; backward pushes their summed gradients. ``rule`` / ``lr``
    default to the optimizer passed to fleet.distributed_optimizer."""

    def __init__(self, size, name=None, padding_idx=None, entry=None, rule=None, lr=None, init="uniform",
                 init_range=None, seed=0):
        super().__init__()
        self.dim = int(size[-1])
        self.table_name = name or f"sparse_embedding_{self.dim}"
        self.padding_idx = padding_idx
        cfg = {"entry": _entry_cfg(entry), "init": init, "seed": int(seed)}
        cfg["init_range"] = float(init_range) if init_range is not None else 1.0 / max(self.dim, 1) ** 0.5
        if rule is not None:
            cfg["rule"] = rule
        if lr is not None:
            cfg["lr"] = float(lr)
        self._cfg = cfg

    def forward(self, ids, show=None, click=None):
        t = ids._t if isinstance(ids, Tensor) else torch.as_tensor(ids)
        sh = None if show is None else (show._t if isinstance(show, Tensor) else torch.as_tensor(show))
        ck = None if click is None else (click._t if isinstance(click, Tensor) else torch.as_tensor(click))
        return _wrap(_ps.sparse_lookup(t.long(), self.table_name, self.dim, training=self.training,
                                       padding_idx=self.padding_idx, cfg=self._cfg, shows=sh, clicks=ck))


class PsOptimizer:
    """fleet.distributed_optimizer(...) in parameter-server mode: ``step()`` pushes dense gradients to the
    servers and pulls the updated values (sync: after every trainer's gradient for this step was averaged;
    async: whatever version is current). The wrapped optimizer's class and learning rate pick the servers'
    update rule."""

    def __init__(self, optimizer, runtime):
        self._opt = optimizer
        self._rt = runtime
        rule = _RULE_OF.get(type(optimizer).__name__, "sgd")
        lr = float(optimizer.get_lr())
        runtime.sparse_rule = {"rule": "adagrad" if rule == "sgd" and type(optimizer).__name__ == "Adagrad"
                               else rule, "lr": lr}
        runtime.dense_rule = {"rule": rule if rule != "adagrad" else "sgd", "lr": lr}
        self._registered = False

    def _params(self):
        return [p for p in self._opt._parameter_list if not getattr(p, "stop_gradient", False)]

    def step(self):
        if not self._registered:
            self._rt.register_dense(self._params())
            self._registered = True
        self._rt.dense_step(self._params())

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        loss.backward()
        self.step()
        return None, None

    def clear_grad(self, set_to_zero=True):
        self._opt.clear_grad(set_to_zero) if set_to_zero is not True else self._opt.clear_grad()

    def __getattr__(self, k):
        return getattr(self._opt, k)
