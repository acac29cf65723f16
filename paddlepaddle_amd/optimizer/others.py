"""SGD, Momentum, Adamax, Adagrad, Adadelta, RMSProp, Lamb, NAdam, RAdam, ASGD, Rprop, LBFGS.
Reference: python/paddle/optimizer/{sgd,momentum,adamax,adagrad,adadelta,rmsprop,lamb,nadam,radam,asgd,
rprop,lbfgs}.py."""
from __future__ import annotations

import math

import torch

from ..framework.grad_mode import no_grad
from ..framework.tensor import _wrap
from .optimizer import Optimizer


class _PerParam(Optimizer):
    def _prep(self, group, p):
        master = self._master(p)
        w = master if master is not None else p._t.detach()
        g = p._t.grad.float() if w.dtype == torch.float32 else p._t.grad
        g = self._regularized_grad(p, g, group)
        lr = self._group_lr(group, p)
        return master, w, g, lr

    def _fin(self, p, master):
        if master is not None:
            p._t.detach().copy_(master)


class _HostLrCapture:
    """SGD / Momentum steps keep no step counters; their learning rate is a kernel argument, so a captured step
    is valid while the learning rate is a constant float and unchanged since the capture (an LRScheduler, or a
    set_lr() after capture, makes the Executor re-run eagerly / re-capture)."""

    def _graph_capturable(self):
        from .lr import LRScheduler
        return not isinstance(self._learning_rate, LRScheduler) and \
            not any(isinstance(g.get("learning_rate"), LRScheduler) for g in self._param_groups)

    def _graph_replay_valid(self, captured_lr):
        return self.get_lr() == captured_lr


class SGD(_HostLrCapture, _PerParam):
    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None,
                 multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        w.add_(g.to(w.dtype), alpha=-lr)
        self._fin(p, master)


class Momentum(_HostLrCapture, _PerParam):
    _acc_names = ("velocity",)

    def __init__(self, learning_rate=0.001, momentum=0.9, parameters=None, use_nesterov=False, weight_decay=None,
                 grad_clip=None, multi_precision=False, rescale_grad=1.0, use_multi_tensor=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._momentum, self._nesterov, self._rescale = momentum, use_nesterov, rescale_grad

    def _update_group(self, group, params):
        """On a HIP device every fp32 (or fp32-master) parameter of the group is updated by one
        multi-tensor launch (csrc/kernels/adamw.hip momentum_multi_k): L2 decay, velocity, the
        parameter and its bf16 shadow in one pass. Others take the per-tensor path."""
        from ..ops import _loader as L
        fused, rest = [], []
        if L.hip_enabled_for(params[0]._t) and L.has("pa_momentum_multi"):
            for p in params:
                reg = self._regularizer_for(p, group)
                ok_reg = reg is None or type(reg).__name__ == "L2Decay"
                ok_dt = p._t.dtype == torch.float32 or self._multi_precision
                (fused if ok_reg and ok_dt and p._t.grad.dtype in L._DT else rest).append(p)
        else:
            rest = params
        if fused:
            self._fused(group, fused)
        for p in rest:
            self._update_param(group, p)

    def _fused(self, group, params):
        from ..ops import _loader as L
        from ..ops import optim as _opt
        from .adam import _f2i
        masters = [self._master(p) for p in params]
        fp32 = [m if m is not None else p._t.detach() for p, m in zip(params, masters)]
        grads = [p._t.grad for p in params]
        key = (tuple(t.data_ptr() for t in fp32), tuple(g.data_ptr() for g in grads))
        tabs = self.__dict__.setdefault("_mt_tables", {})
        tab = tabs.get(id(group))
        if tab is None or tab[0] != key:
            rows, items = [], []
            for i, (w, g, m, p) in enumerate(zip(fp32, grads, masters, params)):
                vel = self._acc("velocity", p)
                reg = self._regularizer_for(p, group)
                lr_mult = p.optimize_attr.get("learning_rate", 1.0) if hasattr(p, "optimize_attr") else 1.0
                ldt = 3 if m is None else L._DT[p._t.dtype]
                rows.append([w.data_ptr(), g.data_ptr(), vel.data_ptr(), 0, 0 if m is None else p._t.data_ptr(),
                             w.numel(), L._DT[g.dtype] | (ldt << 8), _f2i(reg._coeff if reg is not None else 0.0),
                             _f2i(lr_mult)])
                for s0 in range(0, w.numel(), _opt._CHUNK):
                    items.append([i, s0])
            dev = fp32[0].device
            t_rows, h_rows = _opt.device_table(rows, dev)
            t_items, h_items = _opt.device_table(items, dev)
            tab = (key, t_rows, t_items, len(items), fp32, grads, (h_rows, h_items))
            tabs[id(group)] = tab
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                self.__dict__.setdefault("_graph_hosts", []).append(tab[6])  # read by every replay
        _, t_rows, t_items, n_items = tab[:4]
        lr = self._group_lr(group, None)
        mu = group.get("momentum", self._momentum)
        L.call("pa_momentum_multi", L.ptr(t_rows), L.ptr(t_items), n_items,
               L.ptr(getattr(self, "_inv_scale_tensor", None)), float(lr), float(mu), float(self._rescale),
               int(bool(self._nesterov)), L.stream_ptr())

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        g = g.to(w.dtype) * self._rescale
        v = self._acc("velocity", p, dtype=w.dtype)
        mu = group.get("momentum", self._momentum)
        v.mul_(mu).add_(g)
        if self._nesterov:
            w.add_(g + mu * v, alpha=-lr)
        else:
            w.add_(v, alpha=-lr)
        self._fin(p, master)


class Adamax(_PerParam):
    _acc_names = ("moment", "inf_norm", "beta1_pow_acc")

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-08, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps = beta1, beta2, epsilon

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        m = self._acc("moment", p)
        u = self._acc("inf_norm", p)
        bp = self._acc("beta1_pow_acc", p, init=1.0, shape=[1])
        bp.mul_(self._b1)
        m.mul_(self._b1).add_(g, alpha=1 - self._b1)
        torch.maximum(u * self._b2, g.abs() + self._eps, out=u)
        w.addcdiv_(m, u, value=-lr / (1 - bp.item()))
        self._fin(p, master)


class Adagrad(_PerParam):
    _acc_names = ("moment",)

    def __init__(self, learning_rate, epsilon=1e-06, parameters=None, weight_decay=None, grad_clip=None,
                 name=None, initial_accumulator_value=0.0, multi_precision=False):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._eps, self._init = epsilon, initial_accumulator_value

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        m = self._acc("moment", p, init=self._init)
        m.addcmul_(g, g)
        w.addcdiv_(g, m.sqrt().add_(self._eps), value=-lr)
        self._fin(p, master)


class Adadelta(_PerParam):
    _acc_names = ("avg_squared_grad", "avg_squared_update")

    def __init__(self, learning_rate=0.001, epsilon=1e-06, rho=0.95, parameters=None, weight_decay=None,
                 grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._eps, self._rho = epsilon, rho

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        sg = self._acc("avg_squared_grad", p)
        su = self._acc("avg_squared_update", p)
        sg.mul_(self._rho).addcmul_(g, g, value=1 - self._rho)
        upd = -torch.sqrt((su + self._eps) / (sg + self._eps)) * g
        su.mul_(self._rho).addcmul_(upd, upd, value=1 - self._rho)
        w.add_(upd, alpha=lr)
        self._fin(p, master)


class RMSProp(_PerParam):
    _acc_names = ("momentum", "mean_square", "mean_grad")

    def __init__(self, learning_rate, rho=0.95, epsilon=1e-06, momentum=0.0, centered=False, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._rho, self._eps, self._mom, self._centered = rho, epsilon, momentum, centered

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        ms = self._acc("mean_square", p)
        mom = self._acc("momentum", p)
        ms.mul_(self._rho).addcmul_(g, g, value=1 - self._rho)
        if self._centered:
            mg = self._acc("mean_grad", p)
            mg.mul_(self._rho).add_(g, alpha=1 - self._rho)
            denom = (ms - mg * mg + self._eps).sqrt()
        else:
            denom = (ms + self._eps).sqrt()
        mom.mul_(self._mom).addcdiv_(g, denom, value=lr)
        w.sub_(mom)
        self._fin(p, master)


class Lamb(_PerParam):
    _acc_names = ("moment1", "moment2", "beta1_pow_acc", "beta2_pow_acc")

    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-06,
                 parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None, multi_precision=False,
                 always_adapt=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name, multi_precision)
        self._wd, self._b1, self._b2, self._eps = lamb_weight_decay, beta1, beta2, epsilon
        self._exclude = exclude_from_weight_decay_fn
        self._always_adapt = always_adapt

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        m = self._acc("moment1", p)
        v = self._acc("moment2", p)
        b1p = self._acc("beta1_pow_acc", p, init=1.0, shape=[1])
        b2p = self._acc("beta2_pow_acc", p, init=1.0, shape=[1])
        b1p.mul_(self._b1)
        b2p.mul_(self._b2)
        m.mul_(self._b1).add_(g, alpha=1 - self._b1)
        v.mul_(self._b2).addcmul_(g, g, value=1 - self._b2)
        mh = m / (1 - b1p)
        vh = v / (1 - b2p)
        wd = 0.0 if (self._exclude is not None and self._exclude(p)) else self._wd
        r = mh / (vh.sqrt() + self._eps) + wd * w
        wn = w.norm()
        rn = r.norm()
        trust = torch.where((wn > 0) & (rn > 0), wn / rn, torch.ones_like(wn)) if (wd or self._always_adapt) \
            else torch.ones_like(wn)
        w.sub_(lr * trust * r)
        self._fin(p, master)


class NAdam(_PerParam):
    _acc_names = ("moment1", "moment2", "mu_product")

    def __init__(self, learning_rate=0.002, beta1=0.9, beta2=0.999, epsilon=1.0e-8, momentum_decay=0.004,
                 parameters=None, weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps, self._md = beta1, beta2, epsilon, momentum_decay
        self._steps = {}

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        t = self._steps.get(id(p), 0) + 1
        self._steps[id(p)] = t
        m = self._acc("moment1", p)
        v = self._acc("moment2", p)
        mp = self._acc("mu_product", p, init=1.0, shape=[1])
        mu = self._b1 * (1 - 0.5 * 0.96 ** (t * self._md))
        mu1 = self._b1 * (1 - 0.5 * 0.96 ** ((t + 1) * self._md))
        mp.mul_(mu)
        m.mul_(self._b1).add_(g, alpha=1 - self._b1)
        v.mul_(self._b2).addcmul_(g, g, value=1 - self._b2)
        denom = (v / (1 - self._b2 ** t)).sqrt() + self._eps
        mpv = mp.item()
        w.addcdiv_(g, denom, value=-lr * (1 - mu) / (1 - mpv))
        w.addcdiv_(m, denom, value=-lr * mu1 / (1 - mpv * mu1))
        self._fin(p, master)


class RAdam(_PerParam):
    _acc_names = ("moment1", "moment2")

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1.0e-8, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps = beta1, beta2, epsilon
        self._steps = {}

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        t = self._steps.get(id(p), 0) + 1
        self._steps[id(p)] = t
        m = self._acc("moment1", p)
        v = self._acc("moment2", p)
        m.mul_(self._b1).add_(g, alpha=1 - self._b1)
        v.mul_(self._b2).addcmul_(g, g, value=1 - self._b2)
        mh = m / (1 - self._b1 ** t)
        rho_inf = 2 / (1 - self._b2) - 1
        rho_t = rho_inf - 2 * t * self._b2 ** t / (1 - self._b2 ** t)
        if rho_t > 5:
            lt = math.sqrt(1 - self._b2 ** t) / (v.sqrt() + self._eps)
            rt = math.sqrt((rho_t - 4) * (rho_t - 2) * rho_inf / ((rho_inf - 4) * (rho_inf - 2) * rho_t))
            w.add_(mh * lt * rt, alpha=-lr)
        else:
            w.add_(mh, alpha=-lr)
        self._fin(p, master)


class ASGD(_PerParam):
    _acc_names = ("d", "y", "m")

    def __init__(self, learning_rate=0.001, batch_num=1, parameters=None, weight_decay=None, grad_clip=None,
                 multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._n = batch_num
        self._idx = {}

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        ys = self._accumulators["ys"].setdefault(id(p), torch.zeros((self._n,) + tuple(w.shape), device=w.device))
        d = self._acc("d", p)
        i = self._idx.get(id(p), 0)
        cnt = self._accumulators["cnt"].setdefault(id(p), [0])
        d.sub_(ys[i]).add_(g)
        ys[i].copy_(g)
        cnt[0] = min(cnt[0] + 1, self._n)
        self._idx[id(p)] = (i + 1) % self._n
        w.add_(d / cnt[0], alpha=-lr)
        self._fin(p, master)


class Rprop(_PerParam):
    _acc_names = ("prev", "learning_rate")

    def __init__(self, learning_rate=0.001, learning_rate_range=(1e-5, 50), parameters=None, etas=(0.5, 1.2),
                 grad_clip=None, multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name, multi_precision)
        self._range, self._etas = learning_rate_range, etas

    def _update_param(self, group, p):
        master, w, g, lr = self._prep(group, p)
        prev = self._acc("prev", p)
        lrs = self._acc("learning_rate", p, init=lr)
        s = g * prev
        lrs.copy_(torch.where(s > 0, lrs * self._etas[1], torch.where(s < 0, lrs * self._etas[0], lrs)))
        lrs.clamp_(self._range[0], self._range[1])
        g = torch.where(s < 0, torch.zeros_like(g), g)
        w.sub_(torch.sign(g) * lrs)
        prev.copy_(g)
        self._fin(p, master)


class LBFGS(Optimizer):
    """Limited-memory BFGS with optional strong-Wolfe line search (closure-based step)."""

    def __init__(self, learning_rate=1.0, max_iter=20, max_eval=None, tolerance_grad=1e-07,
                 tolerance_change=1e-09, history_size=100, line_search_fn=None, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        import torch.optim as _to
        self._torch_params = [p._t for p in self._parameter_list]
        self._impl = _to.LBFGS(self._torch_params, lr=learning_rate, max_iter=max_iter, max_eval=max_eval,
                               tolerance_grad=tolerance_grad, tolerance_change=tolerance_change,
                               history_size=history_size, line_search_fn=line_search_fn)

    def step(self, closure):
        from ..ops.linear import bump_weight_epoch

        def _c():
            bump_weight_epoch()  # line search evaluates the closure at moved weights
            with torch.enable_grad():
                for t in self._torch_params:
                    t.grad = None
                loss = closure()
            return loss._t if hasattr(loss, "_t") else loss
        r = self._impl.step(_c)
        return _wrap(r) if isinstance(r, torch.Tensor) else r
