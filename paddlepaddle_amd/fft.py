"""paddle.fft (rocFFT via ATen). Reference: python/paddle/fft.py."""
from __future__ import annotations

import torch

from .framework.tensor import _wrap
from .framework.place import _get_torch_device
from .tensor._helpers import T, dtype_arg


def _mk(fn, multi=False):
    if multi:
        def op(x, s=None, axes=None, norm="backward", name=None):
            kw = {"s": s, "norm": norm}
            if axes is not None:
                kw["dim"] = axes
            return _wrap(fn(T(x), **kw))
    else:
        def op(x, n=None, axis=-1, norm="backward", name=None):
            return _wrap(fn(T(x), n=n, dim=axis, norm=norm))
    return op


fft, ifft, rfft, irfft, hfft, ihfft = (_mk(f) for f in (torch.fft.fft, torch.fft.ifft, torch.fft.rfft,
                                                          torch.fft.irfft, torch.fft.hfft, torch.fft.ihfft))
fftn, ifftn, rfftn, irfftn, hfftn, ihfftn = (_mk(f, True) for f in (torch.fft.fftn, torch.fft.ifftn, torch.fft.rfftn,
                                                                      torch.fft.irfftn, torch.fft.hfftn,
                                                                      torch.fft.ihfftn))


def _mk2(fn):
    def op(x, s=None, axes=(-2, -1), norm="backward", name=None):
        return _wrap(fn(T(x), s=s, dim=axes, norm=norm))
    return op


fft2, ifft2, rfft2, irfft2, hfft2, ihfft2 = (_mk2(f) for f in (torch.fft.fft2, torch.fft.ifft2, torch.fft.rfft2,
                                                               torch.fft.irfft2, torch.fft.hfft2, torch.fft.ihfft2))


def fftfreq(n, d=1.0, dtype=None, name=None):
    return _wrap(torch.fft.fftfreq(n, d, dtype=dtype_arg(dtype) or torch.float32, device=_get_torch_device()))


def rfftfreq(n, d=1.0, dtype=None, name=None):
    return _wrap(torch.fft.rfftfreq(n, d, dtype=dtype_arg(dtype) or torch.float32, device=_get_torch_device()))


def fftshift(x, axes=None, name=None):
    return _wrap(torch.fft.fftshift(T(x), axes))


def ifftshift(x, axes=None, name=None):
    return _wrap(torch.fft.ifftshift(T(x), axes))
