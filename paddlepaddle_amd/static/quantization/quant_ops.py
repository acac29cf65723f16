"""Quantization ops recorded into static programs (resolvable by name when a saved program is loaded:
static/program.py _resolve accepts the paddlepaddle_amd.static namespace)."""
from __future__ import annotations

import torch


def _qmax(bits):
    return float(2 ** (int(bits) - 1) - 1)


def fake_quant_act(x, scale, bits):
    """Inference quant-dequant with a calibrated scale (round to nearest, clip)."""
    s = max(float(scale), 1e-8)
    q = _qmax(bits)
    return torch.round(x / s * q).clamp(-q, q) * (s / q)


class _STEActQuant(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, state, moving_rate, bits, training):
        cur = x.detach().abs().max().float()
        if training:
            with torch.no_grad():
                if float(state[1]) == 0.0:          # first step: no history
                    state[0].copy_(cur)
                else:
                    state[0].mul_(moving_rate).add_((1 - moving_rate) * cur)
                state[1].add_(1.0)
        s = state[0].clamp_min(1e-8).to(x.dtype)
        q = _qmax(bits)
        return torch.round(x / s * q).clamp(-q, q) * (s / q)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None, None


def qat_fake_quant_act(x, state, moving_rate, bits):
    """QAT activation fake quant: moving-average abs-max scale kept in ``state`` ([scale, steps]),
    straight-through gradient."""
    return _STEActQuant.apply(x, state, float(moving_rate), int(bits), torch.is_grad_enabled())


class _STEWeightQuant(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w, axis, bits):
        q = _qmax(bits)
        a = w.detach().abs()
        if axis is None:
            s = a.max()
        else:
            red = [i for i in range(w.dim()) if i != axis % w.dim()]
            s = a.amax(dim=red, keepdim=True)
        s = s.clamp_min(1e-8)
        return torch.round(w / s * q).clamp(-q, q) * (s / q)

    @staticmethod
    def backward(ctx, g):
        return g, None, None


def qat_fake_quant_weight(w, axis, bits):
    """QAT weight fake quant (per-tensor when axis is None, else per channel along axis), STE gradient."""
    return _STEWeightQuant.apply(w, None if axis is None else int(axis), int(bits))
