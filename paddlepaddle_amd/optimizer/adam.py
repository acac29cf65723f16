"""Adam / AdamW. Reference: python/paddle/optimizer/{adam,adamw}.py, phi fused_adam_kernel.cu.

On a HIP device every parameter group is updated by ONE multi-tensor kernel launch
(ops.optim / csrc/kernels/adamw.hip): fp32 moments, optional fp32 master weights with the
bf16/fp16 parameter rewritten in the same pass, per-tensor weight-decay and lr multipliers in
the device table.
"""
from __future__ import annotations

import struct

import torch

from .lr import LRScheduler

from ..ops import _loader as L
from ..ops import optim as _opt
from .optimizer import Optimizer


def _f2i(x):
    return struct.unpack("<i", struct.pack("<f", float(x)))[0]


class Adam(Optimizer):
    _acc_names = ("moment1", "moment2", "beta1_pow_acc", "beta2_pow_acc")
    _decoupled = False

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-08, parameters=None,
                 weight_decay=None, grad_clip=None, lazy_mode=False, multi_precision=False, use_multi_tensor=False,
                 amsgrad=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._beta1, self._beta2, self._epsilon = beta1, beta2, epsilon
        self._amsgrad = amsgrad
        self._tables = {}
        self._param_step = {}

    def _coeff_for(self, group, p):
        return 0.0

    def _apply_clip(self):
        """Global-norm clipping folded into the fused update: the clip coefficient stays a device
        scalar that the AdamW kernel multiplies into every gradient it reads (no separate pass over
        the gradients). Other clips, or parameters that take the per-tensor path, scale explicitly."""
        self._clip_coef = None
        clip = self._grad_clip
        from ..nn.clip import ClipGradByGlobalNorm
        ps = [p for p in self._parameter_list if p._t.grad is not None]
        if (isinstance(clip, ClipGradByGlobalNorm) and ps and all(getattr(p, "need_clip", True) for p in ps)
                and L.hip_enabled_for(ps[0]._t) and L.has("pa_adamw_multi") and not self._amsgrad):
            self._clip_coef = clip._coef(ps)
            return
        super()._apply_clip()

    def _hyper(self, group):
        b1 = group.get("beta1", self._beta1)
        b2 = group.get("beta2", self._beta2)
        eps = group.get("epsilon", self._epsilon)
        return float(b1), float(b2), float(eps)

    def _update_group(self, group, params):
        b1, b2, eps = self._hyper(group)
        lr = self._group_lr(group)
        steps = []
        for p in params:
            s = self._param_step.get(id(p), 0) + 1
            self._param_step[id(p)] = s
            steps.append(s)
        dev_ok = L.hip_enabled_for(params[0]._t) and L.has("pa_adamw_multi") and not self._amsgrad
        same_step = all(s == steps[0] for s in steps)
        if dev_ok and same_step and (self._decoupled or not self._has_l2(group, params)):
            self._fused(group, params, lr, b1, b2, eps, steps[0])
            return
        self._host_path = True  # bias correction / lr passed as host floats: not replayable from a graph
        coef = getattr(self, "_clip_coef", None)
        if coef is not None:  # deferred clip, but this group takes the per-tensor path
            torch._foreach_mul_([p._t.grad for p in params], coef)
        for p, s in zip(params, steps):
            self._single(group, p, lr, b1, b2, eps, s)

    def _has_l2(self, group, params):
        return self.regularization is not None or "weight_decay" in group or \
            any(getattr(p, "regularizer", None) is not None for p in params)

    def _single(self, group, p, lr, b1, b2, eps, step):
        master = self._master(p)
        w = master if master is not None else p._t.detach()
        g = p._t.grad.float()
        if not self._decoupled:
            g = self._regularized_grad(p, g, group)
        m = self._acc("moment1", p)
        v = self._acc("moment2", p)
        plr = lr * (p.optimize_attr.get("learning_rate", 1.0) if hasattr(p, "optimize_attr") else 1.0)
        coeff = self._coeff_for(group, p)
        if coeff:
            w.mul_(1.0 - plr * coeff)
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        if self._amsgrad:
            vm = self._acc("moment2_max", p)
            torch.maximum(vm, v, out=vm)
            denom = (vm / bc2).sqrt_().add_(eps)
        else:
            denom = (v / bc2).sqrt_().add_(eps)
        w.addcdiv_(m, denom, value=-plr / bc1)
        if master is not None:
            p._t.detach().copy_(master)
        self._acc("beta1_pow_acc", p, shape=[1]).fill_(b1 ** step)
        self._acc("beta2_pow_acc", p, shape=[1]).fill_(b2 ** step)

    def _fused(self, group, params, lr, b1, b2, eps, step):
        masters = [self._master(p) for p in params]
        fp32 = [m if m is not None else p._t.detach() for p, m in zip(params, masters)]
        grads = [p._t.grad for p in params]
        key = (id(group), tuple(t.data_ptr() for t in fp32), tuple(g.data_ptr() for g in grads))
        tab = self._tables.get(id(group))
        if tab is None or tab[0] != key:
            ms = [self._acc("moment1", p) for p in params]
            vs = [self._acc("moment2", p) for p in params]
            lowps = [p._t.detach() if m is not None else None for p, m in zip(params, masters)]
            rows, items = [], []
            for i, (w, g, m, v, lp, p) in enumerate(zip(fp32, grads, ms, vs, lowps, params)):
                n = w.numel()
                gdt = L._DT[g.dtype]
                ldt = 3 if lp is None else L._DT[lp.dtype]
                lr_mult = p.optimize_attr.get("learning_rate", 1.0) if hasattr(p, "optimize_attr") else 1.0
                rows.append([w.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
                             0 if lp is None else lp.data_ptr(), n, gdt | (ldt << 8),
                             _f2i(self._coeff_for(group, p)), _f2i(lr_mult)])
                for s in range(0, n, _opt._CHUNK):
                    items.append([i, s])
            dev = fp32[0].device
            t_rows, h_rows = _opt.device_table(rows, dev)
            t_items, h_items = _opt.device_table(items, dev)
            tab = (key, t_rows, t_items, len(items), fp32, grads, (h_rows, h_items))
            self._tables[id(group)] = tab
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                self.__dict__.setdefault("_graph_hosts", []).append(tab[6])  # read by every replay
        _, t_rows, t_items, n_items = tab[:4]
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        inv_scale = getattr(self, "_inv_scale_tensor", None)
        coef = getattr(self, "_clip_coef", None)
        if coef is not None:
            inv_scale = coef if inv_scale is None else (coef * inv_scale.reshape(())).reshape(())
        hyper = None
        if fp32[0].is_cuda:
            # the device copy of {lr, beta1^t, beta2^t} is created on the first (eager) step and advanced by every
            # step, so a step captured later into a hipGraph starts from the right powers; eager steps still pass
            # host floats, captured ones read the device copy
            h = self._graph_hyper(group, fp32[0].device, lr, b1, b2, step)
            L.call("pa_adam_hyper_step", L.ptr(h), float(b1), float(b2), L.stream_ptr())
            if torch.cuda.is_current_stream_capturing():
                hyper = h
        L.call("pa_adamw_multi", L.ptr(t_rows), L.ptr(t_items), n_items, L.ptr(inv_scale), float(lr), float(b1),
               float(b2), float(eps), 0.0, float(bc1), float(bc2), L.ptr(hyper), L.stream_ptr())
        self._last_step = step

    def _graph_hyper(self, group, dev, lr, b1, b2, step):
        """Device-resident {lr, beta1^t, beta2^t} of a group whose step is being captured into a hipGraph.
        The captured step advances the beta powers on the device before the update (like the reference's
        beta1_pow / beta2_pow accumulators), so every replay applies its own bias correction; the learning rate
        lives in hyper[0], which the LR scheduler rewrites on each scheduler.step() (and set_lr does too)."""
        hs = self.__dict__.setdefault("_graph_hypers", {})
        h = hs.get(id(group))
        if h is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("capture an optimizer step only after an eager warm-up step (the device "
                                   "hyper-parameter copy is created there)")
            h = torch.tensor([float(lr), float(b1) ** (step - 1), float(b2) ** (step - 1)], dtype=torch.float32,
                             device=dev)
            hs[id(group)] = h
            base = self.get_lr()
            ratio = float(lr) / base if base else 1.0
            if isinstance(self._learning_rate, LRScheduler):
                self._learning_rate._register_device_lr(h, ratio)
            self.__dict__.setdefault("_graph_lr_sinks", []).append((h, ratio))
        return h

    # hipGraph capture: the fused update reads lr and the beta powers from a device copy that the captured step
    # advances itself (_graph_hyper), so replays are exact; the host step counters are advanced per replay here
    # so state_dict() / a later eager step see the true step.
    def _graph_capturable(self):
        return not self._amsgrad and not getattr(self, "_host_path", False)

    def _graph_host_state(self):
        st = super()._graph_host_state()
        st["_param_step"] = dict(self._param_step)
        st["_last_step"] = getattr(self, "_last_step", None)
        return st

    def _graph_restore_host_state(self, state):
        super()._graph_restore_host_state(state)
        self._param_step = dict(state["_param_step"])
        self._last_step = state["_last_step"]

    def _graph_replayed(self, before, after):
        super()._graph_replayed(before, after)
        b, a = before["_param_step"], after["_param_step"]
        for k, s in a.items():
            d = s - b.get(k, 0)
            if d:
                self._param_step[k] = self._param_step.get(k, 0) + d
        if after["_last_step"] is not None:
            self._last_step = (self._last_step or 0) + (after["_last_step"] - (before["_last_step"] or 0))

    def state_dict(self):
        # materialise beta-pow accumulators paddle-style
        for p in self._parameter_list:
            s = self._param_step.get(id(p))
            if s:
                b1, b2, _ = self._hyper({})
                self._acc("beta1_pow_acc", p, shape=[1]).fill_(b1 ** s)
                self._acc("beta2_pow_acc", p, shape=[1]).fill_(b2 ** s)
        return super().state_dict()

    def set_state_dict(self, state_dict):
        super().set_state_dict(state_dict)
        import math
        b1 = self._beta1
        for p in self._parameter_list:
            d = self._accumulators.get("beta1_pow_acc", {})
            if id(p) in d:
                v = float(d[id(p)].reshape(-1)[0].item())
                if 0 < v < 1 and 0 < b1 < 1:
                    self._param_step[id(p)] = int(round(math.log(v) / math.log(b1)))
        self._tables.clear()
        # re-seed the device {lr, beta1^t, beta2^t} copies of a later hipGraph-captured step from the restored
        # step counts (they are otherwise only ever advanced by pa_adam_hyper_step)
        hs = self.__dict__.get("_graph_hypers") or {}
        for group in self._param_groups:
            h = hs.get(id(group))
            if h is None:
                continue
            b1, b2, _ = self._hyper(group)
            st = max((self._param_step.get(id(p), 0) for p in group["params"]), default=0)
            with torch.no_grad():
                h[1:].copy_(torch.tensor([float(b1) ** st, float(b2) ** st], dtype=torch.float32))


class AdamW(Adam):
    _decoupled = True

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None,
                 weight_decay=0.01, lr_ratio=None, apply_decay_param_fun=None, grad_clip=None, lazy_mode=False,
                 multi_precision=False, amsgrad=False, name=None):
        super().__init__(learning_rate, beta1, beta2, epsilon, parameters, None, grad_clip, lazy_mode,
                         multi_precision, False, amsgrad, name)
        self._weight_decay = weight_decay
        self._lr_ratio = lr_ratio
        self._apply_decay_param_fun = apply_decay_param_fun

    def _coeff_for(self, group, p):
        wd = group.get("weight_decay", self._weight_decay)
        if hasattr(wd, "_coeff"):
            wd = wd._coeff
        if self._apply_decay_param_fun is not None and not self._apply_decay_param_fun(p.name):
            return 0.0
        return float(wd or 0.0)

    def _group_lr(self, group, param=None):
        return super()._group_lr(group, None)
