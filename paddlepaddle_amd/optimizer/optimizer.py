"""Optimizer base. Reference: python/paddle/optimizer/optimizer.py.

State naming follows paddle's accumulator convention ("<param>_moment1_0", "master_weights",
"LR_Scheduler") so .pdopt files written here look like paddle's.
"""
from __future__ import annotations

import collections

import numpy as np
import torch

from ..framework.grad_mode import no_grad
from ..framework.tensor import Parameter, Tensor, _wrap
from .lr import LRScheduler


class L2Decay:
    def __init__(self, coeff=0.0):
        self._coeff = float(coeff)
        self._regularization_coeff = self._coeff

    def __call__(self, p, g):
        return g + self._coeff * p


class L1Decay:
    def __init__(self, coeff=0.0):
        self._coeff = float(coeff)
        self._regularization_coeff = self._coeff

    def __call__(self, p, g):
        return g + self._coeff * torch.sign(p)


class Optimizer:
    _acc_names = ()

    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None, name=None,
                 multi_precision=False):
        self._learning_rate = learning_rate
        if parameters is None:
            from ..static import _static_mode
            if not _static_mode.enabled:
                raise ValueError("parameters must be given in dygraph mode (static mode: use minimize)")
            parameters = []  # filled from the program by minimize()
        parameters = list(parameters)
        if parameters and isinstance(parameters[0], dict):
            self._param_groups = []
            for g in parameters:
                gg = dict(g)
                gg["params"] = list(gg["params"])
                self._param_groups.append(gg)
        else:
            self._param_groups = [{"params": parameters}]
        self._parameter_list = [p for g in self._param_groups for p in g["params"]]
        if isinstance(weight_decay, float) or isinstance(weight_decay, int):
            self.regularization = L2Decay(float(weight_decay)) if weight_decay else None
        else:
            self.regularization = weight_decay
        self._grad_clip = grad_clip
        self._multi_precision = multi_precision
        self._accumulators = collections.defaultdict(dict)  # acc name -> {param id: tensor}
        self._master_weights = {}
        self._step_count = 0
        self._name = name
        self.helper = None

    # ------------------------------------------------------------------ lr
    def get_lr(self):
        if isinstance(self._learning_rate, LRScheduler):
            return float(self._learning_rate())
        return float(self._learning_rate)

    def set_lr(self, value):
        if isinstance(self._learning_rate, LRScheduler):
            raise RuntimeError("cannot set_lr when an LRScheduler is used")
        old = float(self._learning_rate)
        self._learning_rate = float(value)
        for h, ratio in self.__dict__.get("_graph_lr_sinks", ()):  # captured steps read lr from the device
            h[0].fill_(float(value) * ratio if old else float(value))

    def set_lr_scheduler(self, scheduler):
        self._learning_rate = scheduler

    def _group_lr(self, group, param=None):
        lr = self.get_lr()
        if "learning_rate" in group:
            lr = lr * group["learning_rate"] if not isinstance(group["learning_rate"], LRScheduler) \
                else float(group["learning_rate"]())
        if param is not None and isinstance(param, Parameter):
            lr = lr * param.optimize_attr.get("learning_rate", 1.0)
        return lr

    # ------------------------------------------------------------------ state
    def _acc(self, name, p, init=0.0, dtype=torch.float32, shape=None):
        d = self._accumulators[name]
        k = id(p)
        if k not in d:
            t = p._t
            if shape is None and type(t) is not torch.Tensor:
                d[k] = torch.full_like(t.detach(), init, dtype=dtype)  # distributed params: same placements
            elif shape is None:
                d[k] = torch.full(t.shape, init, dtype=dtype, device=t.device)
            else:
                d[k] = torch.full(shape, init, dtype=dtype, device=t.device)
        return d[k]

    def _master(self, p):
        """fp32 master copy for low-precision params when multi_precision is on."""
        t = p._t
        if not self._multi_precision or t.dtype == torch.float32:
            return None
        k = id(p)
        if k not in self._master_weights:
            self._master_weights[k] = t.detach().float().clone()
        return self._master_weights[k]

    def state_dict(self):
        sd = collections.OrderedDict()
        for name, d in self._accumulators.items():
            for p in self._parameter_list:
                if id(p) in d:
                    sd[f"{p.name}_{name}_0"] = _wrap(d[id(p)])
        if self._master_weights:
            sd["master_weights"] = {p.name: _wrap(self._master_weights[id(p)]) for p in self._parameter_list
                                    if id(p) in self._master_weights}
        if isinstance(self._learning_rate, LRScheduler):
            sd["LR_Scheduler"] = self._learning_rate.state_dict()
        sd["@step"] = self._step_count
        return sd

    def set_state_dict(self, state_dict):
        if "LR_Scheduler" in state_dict and isinstance(self._learning_rate, LRScheduler):
            self._learning_rate.set_state_dict(state_dict["LR_Scheduler"])
        self._step_count = int(state_dict.get("@step", self._step_count))
        by_name = {p.name: p for p in self._parameter_list}
        for key, v in state_dict.items():
            if key in ("LR_Scheduler", "master_weights", "@step"):
                continue
            for acc in self._acc_names:
                suffix = f"_{acc}_0"
                if key.endswith(suffix) and key[: -len(suffix)] in by_name:
                    p = by_name[key[: -len(suffix)]]
                    src = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
                    self._accumulators[acc][id(p)] = src.to(p._t.device).clone().float() \
                        if src.is_floating_point() else src.to(p._t.device).clone()
        for name, v in state_dict.get("master_weights", {}).items():
            if name in by_name:
                src = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
                self._master_weights[id(by_name[name])] = src.to(by_name[name]._t.device).float().clone()

    set_dict = set_state_dict

    # ------------------------------------------------------------------ step
    def clear_grad(self, set_to_zero=True):
        # DataParallel's flat all-reduce buckets: a bucket may hold parameters of several optimizers (e.g. the
        # generator and discriminator of one wrapped GAN), so a whole-bucket memset is only legal when every
        # parameter in it is ours; otherwise only our own slices are zeroed
        own = {id(p) for p in self._parameter_list}
        whole = {}
        for p in self._parameter_list:
            loc = getattr(p, "_dp_bucket", None)
            if loc is not None and id(loc[0]) not in whole:
                whole[id(loc[0])] = all(id(q) in own for q in loc[0].params)
        zeroed = set()
        for p in self._parameter_list:
            loc = getattr(p, "_dp_bucket", None)
            if loc is not None:
                bucket, j = loc
                v = bucket.view(j)
                if set_to_zero and whole[id(bucket)]:
                    # the grad stays a view of the bucket (releasing it would make the next backward allocate a
                    # fresh gradient that has to be copied back); one memset per bucket
                    if id(bucket) not in zeroed:
                        zeroed.add(id(bucket))
                        bucket.flat.zero_()
                else:
                    v.zero_()  # an unused parameter contributes zeros to the next all-reduce
                if set_to_zero:
                    if p._t.grad is None or p._t.grad.data_ptr() != v.data_ptr():
                        p._t.grad = v
                else:
                    p._t.grad = None  # DataParallel's ready hook folds the next fresh grad back into the bucket
                continue
            if set_to_zero:
                if p._t.grad is not None:
                    p._t.grad.zero_()
            else:
                p._t.grad = None

    clear_gradients = clear_grad

    def _params_with_grad(self, group):
        return [p for p in group["params"] if getattr(p, "trainable", True) and p._t.grad is not None]

    def _apply_clip(self):
        clip = self._grad_clip
        if clip is None:
            return
        ps = [p for p in self._parameter_list if p._t.grad is not None]
        clip._clip_inplace(ps)

    def _regularizer_for(self, p, group):
        reg = getattr(p, "regularizer", None) or group.get("weight_decay_obj", None) or self.regularization
        if "weight_decay" in group and not isinstance(group["weight_decay"], (L1Decay, L2Decay)):
            wd = group["weight_decay"]
            reg = L2Decay(wd) if wd else None
        elif "weight_decay" in group:
            reg = group["weight_decay"]
        return reg

    def _regularized_grad(self, p, g, group):
        reg = self._regularizer_for(p, group)
        if reg is None:
            return g
        return reg(p._t.detach().to(g.dtype), g)

    @no_grad()
    def step(self):
        from ..ops.linear import bump_weight_epoch
        bump_weight_epoch()  # weights change: drop per-step forward-layout weight copies
        self._step_count += 1
        self._apply_clip()
        for group in self._param_groups:
            params = self._params_with_grad(group)
            if params:
                self._update_group(group, params)

    def _update_group(self, group, params):
        for p in params:
            self._update_param(group, p)

    # ------------------------------------------------------------------ hipGraph capture of a step
    # A captured training step (static.Executor with BuildStrategy.allow_cuda_graph_capture) replays only device
    # work: host-side state that the update reads (a learning rate passed as a kernel argument, step counters
    # used for bias correction) is frozen at its capture-time value. An optimizer therefore says whether its
    # step may be captured, and keeps its host bookkeeping in step with the replays.
    def _graph_capturable(self):
        """Whether a step of this optimizer stays correct when replayed from a hipGraph. Default: no."""
        return False

    def _graph_host_state(self):
        """Snapshot of the host-side state a step mutates (restored when a capture fails part-way)."""
        return {"_step_count": self._step_count}

    def _graph_restore_host_state(self, state):
        self._step_count = state["_step_count"]

    def _graph_replayed(self, before, after):
        """Called after every replay of a step captured between host states ``before`` and ``after``: advance
        the host bookkeeping by what the captured step did."""
        self._step_count += after["_step_count"] - before["_step_count"]

    def _graph_replay_valid(self, captured_lr):
        """False when a replay would apply a stale host hyper-parameter (the graph must be re-captured)."""
        return True

    def _update_param(self, group, p):
        raise NotImplementedError

    def _write_back(self, p, master, new_fp32):
        """new_fp32 was computed in-place on master (or p itself)."""
        if master is not None:
            p._t.detach().copy_(master)

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        from ..static import _static_mode
        if _static_mode.enabled:
            from ..static import default_main_program
            default_main_program()._set_optimizer(self, loss)
            return None, None
        loss.backward()
        self.step()
        return None, None

    def backward(self, loss, startup_program=None, parameters=None, no_grad_set=None, callbacks=None):
        loss.backward()
        return [(p, p.grad) for p in self._parameter_list]

    def apply_gradients(self, params_grads):
        for p, g in params_grads:
            if g is not None and p._t.grad is None:
                p._t.grad = g._t
        self.step()
