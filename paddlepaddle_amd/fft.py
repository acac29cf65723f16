"""paddle.fft. Reference: python/paddle/fft.py (every public transform there is one of three kernels,
fft_c2c / fft_r2c / fft_c2r of paddle/phi/kernels/gpu/fft_kernel.cu, plus argument checking and resizing).

Same layering here: this module validates and normalises the paddle arguments (``n`` / ``s`` resizing by zero
padding or truncation, negative / duplicate axes, the three ``norm`` modes) and reduces all 18 transforms to
three primitives that run rocFFT through ATen:

* ``_c2c(x, axes, norm, forward)``     complex -> complex
* ``_r2c(x, axes, norm, forward, onesided)``   real -> half (or full) spectrum
* ``_c2r(x, axes, norm, forward, last)``    half spectrum -> real of length ``last`` on the last axis

``forward`` selects the sign of the exponent and which side of the transform pair ``norm`` scales
("backward": 1 forward / 1/n inverse, "forward": the reverse, "ortho": 1/sqrt(n) both), which is how the
Hermitian transforms are expressed: hfft = c2r with forward=True, ihfft = r2c with forward=False.
"""
from __future__ import annotations

import math

import torch

from .framework.tensor import Tensor, _wrap
from .framework.place import _get_torch_device
from .tensor._helpers import T, dtype_arg

_NORMS = ("backward", "forward", "ortho")


# ---------------------------------------------------------------------------------------------- checks
def _check_norm(norm):
    if norm not in _NORMS:
        raise ValueError(f"Unexpected norm: {norm}. Norm should be forward, backward or ortho")


def _check_n(n, what="n"):
    if n is not None and (not isinstance(n, int) or n <= 0):
        raise ValueError(f"Invalid FFT argument {what}({n}), it should be a positive integer.")


def _norm_axes(x, axes, s, default_all=True):
    """Resolve (axes, s) the way paddle does: axes default to the last len(s) axes (or all axes); negative
    axes wrap; duplicates are an error."""
    nd = x.dim()
    if s is not None:
        s = [int(v) for v in (s._t.tolist() if isinstance(s, Tensor) else s)]
        for v in s:
            _check_n(v, "s")
    if axes is None:
        axes = list(range(nd - len(s), nd)) if s is not None else (list(range(nd)) if default_all else [nd - 1])
    else:
        axes = [int(a) for a in (axes._t.tolist() if isinstance(axes, Tensor) else
                                 (axes if isinstance(axes, (list, tuple)) else [axes]))]
    for a in axes:
        if not -nd <= a < nd:
            raise ValueError(f"Invalid axis {a} for a tensor of rank {nd}")
    axes = [a % nd for a in axes]
    if len(set(axes)) != len(axes):
        raise ValueError(f"Duplicate axes are not allowed: {axes}")
    if s is not None and len(s) != len(axes):
        raise ValueError(f"Length of s ({len(s)}) and length of axes ({len(axes)}) do not match")
    return axes, s


def _resize(t, axes, sizes):
    """Zero-pad or truncate ``t`` to ``sizes`` along ``axes`` (paddle's fft ``n`` / ``s`` semantics)."""
    if sizes is None:
        return t
    for a, n in zip(axes, sizes):
        cur = t.shape[a]
        if n < cur:
            t = t.narrow(a, 0, n)
        elif n > cur:
            pad_shape = list(t.shape)
            pad_shape[a] = n - cur
            t = torch.cat([t, torch.zeros(pad_shape, dtype=t.dtype, device=t.device)], a)
    return t


def _scale(norm, n, forward):
    """Multiplier applied by a transform of total length n in direction `forward` under `norm`."""
    if norm == "ortho":
        return 1.0 / math.sqrt(n)
    if (norm == "backward") != forward:  # backward-inverse or forward-forward
        return 1.0 / n
    return 1.0


def _to_complex(t):
    if t.is_complex():
        return t
    return t.to(torch.complex128 if t.dtype == torch.float64 else torch.complex64)


def _to_real(t):
    if t.is_complex():
        raise TypeError("this transform expects a real input tensor")
    if not t.is_floating_point():
        t = t.to(torch.float32)
    return t


# ---------------------------------------------------------------------------------------------- primitives
def _c2c(t, axes, norm, forward):
    t = _to_complex(t)
    n = math.prod(t.shape[a] for a in axes) if axes else 1
    out = (torch.fft.fftn if forward else torch.fft.ifftn)(t, dim=axes, norm="forward" if not forward else "backward")
    # the call above is unnormalised in both directions ("backward" forward / "forward" inverse)
    sc = _scale(norm, n, forward)
    return out * sc if sc != 1.0 else out


def _r2c(t, axes, norm, forward, onesided=True):
    t = _to_real(t)
    n = math.prod(t.shape[a] for a in axes) if axes else 1
    out = torch.fft.rfftn(t, dim=axes, norm="backward") if onesided else \
        torch.fft.fftn(_to_complex(t), dim=axes, norm="backward")
    if not forward:  # inverse-direction transform of a real signal = conjugate of the forward one
        out = out.conj().resolve_conj()
    sc = _scale(norm, n, forward)
    return out * sc if sc != 1.0 else out


def _c2r(t, axes, norm, forward, last):
    t = _to_complex(t)
    sizes = [t.shape[a] for a in axes[:-1]] + [last]
    n = math.prod(sizes)
    if forward:  # forward-direction transform of a Hermitian signal: inverse of its conjugate
        t = t.conj().resolve_conj()
    out = torch.fft.irfftn(t, s=sizes, dim=axes, norm="forward")  # unnormalised inverse
    sc = _scale(norm, n, forward)
    return out * sc if sc != 1.0 else out


# ---------------------------------------------------------------------------------------------- 1-D
def _one(kind, x, n, axis, norm, forward):
    _check_norm(norm)
    _check_n(n)
    t = T(x)
    axes, _ = _norm_axes(t, [axis], None)
    if kind == "c2c":
        return _wrap(_c2c(_resize(t, axes, [n] if n else None), axes, norm, forward))
    if kind == "r2c":
        return _wrap(_r2c(_resize(_to_real(t), axes, [n] if n else None), axes, norm, forward))
    last = n if n is not None else 2 * (t.shape[axes[0]] - 1)
    if last < 1:
        raise ValueError(f"Invalid number of data points ({last}) specified")
    t = _resize(t, axes, [last // 2 + 1])
    return _wrap(_c2r(t, axes, norm, forward, last))


def fft(x, n=None, axis=-1, norm="backward", name=None):
    return _one("c2c", x, n, axis, norm, True)


def ifft(x, n=None, axis=-1, norm="backward", name=None):
    return _one("c2c", x, n, axis, norm, False)


def rfft(x, n=None, axis=-1, norm="backward", name=None):
    return _one("r2c", x, n, axis, norm, True)


def irfft(x, n=None, axis=-1, norm="backward", name=None):
    return _one("c2r", x, n, axis, norm, False)


def hfft(x, n=None, axis=-1, norm="backward", name=None):
    return _one("c2r", x, n, axis, norm, True)


def ihfft(x, n=None, axis=-1, norm="backward", name=None):
    return _one("r2c", x, n, axis, norm, False)


# ---------------------------------------------------------------------------------------------- n-D
def _many(kind, x, s, axes, norm, forward, default_all=True):
    _check_norm(norm)
    t = T(x)
    axes, s = _norm_axes(t, axes, s, default_all)
    if not axes:
        return _wrap(t.clone())
    if kind == "c2c":
        return _wrap(_c2c(_resize(t, axes, s), axes, norm, forward))
    if kind == "r2c":
        return _wrap(_r2c(_resize(_to_real(t), axes, s), axes, norm, forward))
    last = s[-1] if s is not None else 2 * (t.shape[axes[-1]] - 1)
    if last < 1:
        raise ValueError(f"Invalid number of data points ({last}) specified")
    sizes = (list(s[:-1]) if s is not None else [t.shape[a] for a in axes[:-1]]) + [last // 2 + 1]
    return _wrap(_c2r(_resize(t, axes, sizes), axes, norm, forward, last))


def fftn(x, s=None, axes=None, norm="backward", name=None):
    return _many("c2c", x, s, axes, norm, True)


def ifftn(x, s=None, axes=None, norm="backward", name=None):
    return _many("c2c", x, s, axes, norm, False)


def rfftn(x, s=None, axes=None, norm="backward", name=None):
    return _many("r2c", x, s, axes, norm, True)


def irfftn(x, s=None, axes=None, norm="backward", name=None):
    return _many("c2r", x, s, axes, norm, False)


def hfftn(x, s=None, axes=None, norm="backward", name=None):
    return _many("c2r", x, s, axes, norm, True)


def ihfftn(x, s=None, axes=None, norm="backward", name=None):
    return _many("r2c", x, s, axes, norm, False)


def _check_2d(s, axes):
    if axes is not None and len(axes) != 2:
        raise ValueError(f"Invalid FFT argument axes ({axes}), it should be a sequence of 2 integers.")
    if s is not None and len(s) != 2:
        raise ValueError(f"Invalid FFT argument s ({s}), it should be a sequence of 2 integers.")


def fft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    _check_2d(s, axes)
    return fftn(x, s, axes, norm)


def ifft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    _check_2d(s, axes)
    return ifftn(x, s, axes, norm)


def rfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    _check_2d(s, axes)
    return rfftn(x, s, axes, norm)


def irfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    _check_2d(s, axes)
    return irfftn(x, s, axes, norm)


def hfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    _check_2d(s, axes)
    return hfftn(x, s, axes, norm)


def ihfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    _check_2d(s, axes)
    return ihfftn(x, s, axes, norm)


# ---------------------------------------------------------------------------------------------- helpers
def fftfreq(n, d=1.0, dtype=None, name=None):
    """Sample frequencies [0, 1, ..., n/2-1, -n/2, ..., -1] / (d*n)."""
    dt = dtype_arg(dtype) or torch.get_default_dtype()
    dev = _get_torch_device()
    pos = torch.arange(0, (n - 1) // 2 + 1, device=dev)
    neg = torch.arange(-(n // 2), 0, device=dev)
    return _wrap((torch.cat([pos, neg]).to(dt) / (n * d)).to(dt))


def rfftfreq(n, d=1.0, dtype=None, name=None):
    """Non-negative sample frequencies [0, ..., n//2] / (d*n) of rfft."""
    dt = dtype_arg(dtype) or torch.get_default_dtype()
    return _wrap((torch.arange(0, n // 2 + 1, device=_get_torch_device()).to(dt) / (n * d)).to(dt))


def _shift_axes(t, axes):
    if axes is None:
        return list(range(t.dim()))
    return [int(a) for a in (axes if isinstance(axes, (list, tuple)) else [axes])]


def fftshift(x, axes=None, name=None):
    """Move the zero-frequency term to the centre: roll every axis by floor(n/2)."""
    t = T(x)
    ax = _shift_axes(t, axes)
    return _wrap(torch.roll(t, [t.shape[a] // 2 for a in ax], ax))


def ifftshift(x, axes=None, name=None):
    """Inverse of fftshift: roll by -floor(n/2)."""
    t = T(x)
    ax = _shift_axes(t, axes)
    return _wrap(torch.roll(t, [-(t.shape[a] // 2) for a in ax], ax))


# primitives under paddle's names (paddle.fft exposes them to signal.stft / istft)
def fft_c2c(x, n, axis, norm, forward, name=None):
    t = T(x)
    axes, _ = _norm_axes(t, [axis], None)
    return _wrap(_c2c(_resize(t, axes, [n] if n else None), axes, norm, forward))


def fft_r2c(x, n, axis, norm, forward, onesided, name=None):
    t = T(x)
    axes, _ = _norm_axes(t, [axis], None)
    return _wrap(_r2c(_resize(_to_real(t), axes, [n] if n else None), axes, norm, forward, onesided))


def fft_c2r(x, n, axis, norm, forward, name=None):
    t = T(x)
    axes, _ = _norm_axes(t, [axis], None)
    last = n if n is not None else 2 * (t.shape[axes[0]] - 1)
    return _wrap(_c2r(_resize(t, axes, [last // 2 + 1]), axes, norm, forward, last))


__all__ = ["fft", "ifft", "rfft", "irfft", "hfft", "ihfft", "fft2", "ifft2", "rfft2", "irfft2", "hfft2", "ihfft2",
           "fftn", "ifftn", "rfftn", "irfftn", "hfftn", "ihfftn", "fftfreq", "rfftfreq", "fftshift", "ifftshift"]
