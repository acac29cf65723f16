"""paddle.incubate.layers.nn. Reference: python/paddle/incubate/layers/nn.py (fused_bn_add_act :1092, shuffle_batch
:274, partial_concat :346, partial_sum :426, batch_fc :932, correlation :1003, pow2_decay_with_linear_warmup
:1297; kernels paddle/phi/kernels/gpu/correlation_kernel.cu, batch_fc_kernel.cu,
impl/pow2_decay_with_linear_warmup_kernel_impl.h).

Layer functions create their parameters on each call, as the reference's static layer functions do. The
parameter-server feature ops of that module (fused_seqpool_cvm, search_pyramid_hash, tdm_child, tdm_sampler,
rank_attention, _pull_gpups_sparse, _pull_box_sparse) need the GPUPS / BoxPS sparse tables and raise."""
from __future__ import annotations

import math

import torch

from ...framework.tensor import Tensor, _wrap
from ...nn.layer.layers import create_parameter_tensor


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def fused_bn_add_act(x, y, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None, moving_mean_name=None,
                     moving_variance_name=None, act=None, name=None):
    """act(batch_norm(x) + y) over NHWC x (training statistics), one fused pass (csrc/kernels/bn.hip)."""
    from ...nn import initializer as I
    from ...nn.functional.norm import fused_bn_act
    from ...nn.layer.layers import ParamAttr
    C = _t(x).shape[-1]
    dev = _t(x).device
    w = create_parameter_tensor([C], "float32", param_attr, default_initializer=I.Constant(1.0), device=dev)
    b = create_parameter_tensor([C], "float32", bias_attr, is_bias=True, device=dev)
    mean = create_parameter_tensor([C], "float32", ParamAttr(name=moving_mean_name, initializer=I.Constant(0.0),
                                                             trainable=False), device=dev)
    var = create_parameter_tensor([C], "float32", ParamAttr(name=moving_variance_name, initializer=I.Constant(1.0),
                                                            trainable=False), device=dev)
    return fused_bn_act(x, mean, var, w, b, True, momentum, epsilon, "NHWC", None, act, y)


def shuffle_batch(x, seed=None):
    """Rows (every dim but the last, flattened) in a random order; the last dim stays whole."""
    t = _t(x)
    g = None
    if seed is not None:
        g = torch.Generator(device="cpu").manual_seed(int(_t(seed).item() if hasattr(_t(seed), "item") else seed))
    rows = t.reshape(-1, t.shape[-1])
    perm = torch.randperm(rows.shape[0], generator=g).to(t.device)
    return _wrap(rows[perm].reshape(t.shape))


def _partial(inputs, start_index, length):
    ts = [_t(v) for v in inputs]
    for v in ts:
        if v.dim() != 2:
            raise ValueError("partial_concat / partial_sum take 2-D inputs")
    cols = ts[0].shape[1]
    s = start_index + cols if start_index < 0 else start_index
    e = cols if length < 0 else s + length
    return [v[:, s:e] for v in ts]


def partial_concat(input, start_index=0, length=-1):
    return _wrap(torch.cat(_partial(input, start_index, length), dim=1))


def partial_sum(input, start_index=0, length=-1):
    parts = _partial(input, start_index, length)
    out = parts[0].clone()
    for p in parts[1:]:
        out = out + p
    return _wrap(out)


def batch_fc(input, param_size, param_attr, bias_size, bias_attr, act=None):
    """out[s] = act(input[s] @ W[s] + b[s]) for every slot s: input [S, B, in], W param_size [S, in, out],
    bias bias_size [S, out] (one batched GEMM)."""
    t = _t(input)
    w = create_parameter_tensor(list(param_size), str(t.dtype).replace("torch.", ""), param_attr, device=t.device)
    b = create_parameter_tensor(list(bias_size), str(t.dtype).replace("torch.", ""), bias_attr, is_bias=True,
                                device=t.device)
    wt, bt = _t(w), _t(b)
    out = torch.baddbmm(bt.reshape(bt.shape[0], 1, -1), t, wt)
    if act == "relu":
        out = torch.relu(out)
    elif act is not None:
        out = getattr(torch.nn.functional, act)(out)
    return _wrap(out)


def correlation(x, y, pad_size, kernel_size, max_displacement, stride1, stride2, corr_type_multiply=1):
    """PWC-Net cost volume (reference correlation_kernel.cu): for every displacement (tj, ti) on the stride2 grid,
    the channel dot product of x and y shifted by it, summed over a kernel_size window and divided by
    kernel_size^2 * C, sampled every stride1 pixels from the border max_displacement."""
    a, b = _t(x), _t(y)
    N, C, H, W = a.shape
    kr = (kernel_size - 1) // 2
    dr = max_displacement // stride2
    border = kr + max_displacement
    Hp, Wp = H + 2 * pad_size, W + 2 * pad_size
    OH = math.ceil((Hp - 2 * border) / stride1)
    OW = math.ceil((Wp - 2 * border) / stride1)
    pa = torch.nn.functional.pad(a, [pad_size] * 4)
    pb = torch.nn.functional.pad(b, [pad_size] * 4)
    md = max_displacement
    rows = torch.arange(OH, device=a.device) * stride1 + md
    cols = torch.arange(OW, device=a.device) * stride1 + md
    outs = []
    for tj in range(-dr, dr + 1):
        for ti in range(-dr, dr + 1):
            dy, dx = tj * stride2, ti * stride2
            shifted = torch.zeros_like(pb)
            ys0, ys1 = max(0, -dy), min(Hp, Hp - dy)
            xs0, xs1 = max(0, -dx), min(Wp, Wp - dx)
            shifted[:, :, ys0:ys1, xs0:xs1] = pb[:, :, ys0 + dy:ys1 + dy, xs0 + dx:xs1 + dx]
            prod = (pa * shifted).sum(1, keepdim=True)
            if kr:
                prod = torch.nn.functional.avg_pool2d(prod, kernel_size, 1, kr, count_include_pad=True) * (
                    kernel_size * kernel_size)
            outs.append(prod[:, :, rows][:, :, :, cols])
    return _wrap(torch.cat(outs, 1) / (kernel_size * kernel_size * C))


class _Pow2DecayWithLinearWarmup:
    """Callable learning rate of pow2_decay_with_linear_warmup: each ``step()`` advances it like the kernel."""

    def __init__(self, warmup_steps, total_steps, base_lr, end_lr):
        if warmup_steps > total_steps:
            raise ValueError("warmup_steps cannot be larger than total_steps")
        self.warmup_steps, self.total_steps = int(warmup_steps), int(total_steps)
        self.base_lr, self.end_lr = float(base_lr), float(end_lr)
        self.step_num = 0
        self.last_lr = self.base_lr / self.warmup_steps

    def step(self):
        s = self.step_num = self.step_num + 1
        if s <= self.warmup_steps:
            self.last_lr = s / self.warmup_steps * self.base_lr
        elif s < self.total_steps:
            f = 1 - (s - self.warmup_steps) / (self.total_steps - self.warmup_steps)
            self.last_lr = (self.base_lr - self.end_lr) * f * f + self.end_lr
        else:
            self.last_lr = self.end_lr
        return self.last_lr

    def __call__(self):
        return self.last_lr

    def get_lr(self):
        return self.last_lr


def pow2_decay_with_linear_warmup(warmup_steps, total_steps, base_lr, end_lr, dtype="float32", name=None):
    """Linear warmup to base_lr, then (base_lr - end_lr) * (1 - progress)^2 + end_lr (reference kernel impl). The
    reference returns a persistable static variable advanced by an op; here an LR object with step() / get_lr()
    usable as an optimizer learning_rate in either mode."""
    return _Pow2DecayWithLinearWarmup(warmup_steps, total_steps, base_lr, end_lr)


def _ps_only(name):
    def f(*a, **k):
        raise NotImplementedError(f"paddle.incubate.layers.{name}: a parameter-server (GPUPS / BoxPS) sparse-table "
                                  f"op; this framework's PS (paddle.distributed.ps) does not host those tables")
    f.__name__ = name
    return f


fused_seqpool_cvm = _ps_only("fused_seqpool_cvm")
search_pyramid_hash = _ps_only("search_pyramid_hash")
tdm_child = _ps_only("tdm_child")
tdm_sampler = _ps_only("tdm_sampler")
rank_attention = _ps_only("rank_attention")
_pull_gpups_sparse = _ps_only("_pull_gpups_sparse")
_pull_box_sparse = _ps_only("_pull_box_sparse")
