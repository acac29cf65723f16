"""paddle.signal: frame / overlap_add and the short-time Fourier transform built on them.
Reference: python/paddle/signal.py (frame, overlap_add, stft, istft).

stft = reflect/constant centre padding -> ``frame`` into [batch, n_fft, num_frames] -> window (zero-padded to
n_fft, centred) -> real-to-complex (onesided) or complex-to-complex FFT along the frame axis, ``normalized``
meaning the "ortho" scale. istft inverts it: inverse FFT per frame, window, ``overlap_add`` of the frames and of
the squared window (the NOLA envelope), division by the envelope, trimming of the centre padding / ``length``.
The frame / overlap-add index maps are gathers and index-adds on the device, so the whole transform stays on the
GPU and is differentiable.
"""
from __future__ import annotations

import torch

from .framework.tensor import _wrap
from .tensor._helpers import T
from . import fft as _fft


# ---------------------------------------------------------------------------------------------- framing
def _frame_index(seq_len, frame_length, hop_length, device):
    n_frames = 1 + (seq_len - frame_length) // hop_length
    return (torch.arange(frame_length, device=device)[:, None] +
            hop_length * torch.arange(n_frames, device=device)[None, :])  # [frame_length, n_frames]


def frame(x, frame_length, hop_length, axis=-1, name=None):
    """Slice a signal into overlapping frames. axis=-1: [..., seq] -> [..., frame_length, num_frames];
    axis=0: [seq, ...] -> [num_frames, frame_length, ...]."""
    t = T(x)
    if axis not in (0, -1):
        raise ValueError(f"Unexpected axis: {axis}. It should be 0 or -1.")
    if not isinstance(frame_length, int) or frame_length <= 0:
        raise ValueError(f"Unexpected frame_length: {frame_length}. It should be an positive integer.")
    if not isinstance(hop_length, int) or hop_length <= 0:
        raise ValueError(f"Unexpected hop_length: {hop_length}. It should be an positive integer.")
    seq_len = t.shape[axis]
    if frame_length > seq_len:
        raise ValueError(f"Attribute frame_length should be less equal than sequence length, "
                         f"but got ({frame_length}) > ({seq_len}).")
    idx = _frame_index(seq_len, frame_length, hop_length, t.device)
    if axis == -1:
        return _wrap(t[..., idx])                                   # [..., frame_length, n_frames]
    out = t[idx.t()]                                                # [n_frames, frame_length, ...]
    return _wrap(out)


def overlap_add(x, hop_length, axis=-1, name=None):
    """Sum overlapping frames back into a signal. axis=-1: [..., frame_length, num_frames] -> [..., seq];
    axis=0: [num_frames, frame_length, ...] -> [seq, ...]; seq = (num_frames - 1) * hop + frame_length."""
    t = T(x)
    if axis not in (0, -1):
        raise ValueError(f"Unexpected axis: {axis}. It should be 0 or -1.")
    if not isinstance(hop_length, int) or hop_length <= 0:
        raise ValueError(f"Unexpected hop_length: {hop_length}. It should be an positive integer.")
    if axis == 0:
        t = t.movedim(0, -1).movedim(0, -2)  # [frame_length... ] -> [..., frame_length, n_frames]
    frame_length, n_frames = t.shape[-2], t.shape[-1]
    seq_len = (n_frames - 1) * hop_length + frame_length
    idx = (torch.arange(frame_length, device=t.device)[:, None] +
           hop_length * torch.arange(n_frames, device=t.device)[None, :]).reshape(-1)
    lead = t.shape[:-2]
    src = t.reshape(*lead, frame_length * n_frames)
    out = torch.zeros(*lead, seq_len, dtype=t.dtype, device=t.device).index_add(-1, idx, src)
    if axis == 0:
        out = out.movedim(-1, 0)
    return _wrap(out)


# ---------------------------------------------------------------------------------------------- STFT
def _padded_window(window, win_length, n_fft, dtype, device):
    if window is None:
        w = torch.ones(win_length, dtype=dtype, device=device)
    else:
        w = T(window)
        if w.dim() != 1 or w.shape[0] != win_length:
            raise ValueError(f"expected a 1D window tensor of size equal to win_length({win_length}), "
                             f"but got window with shape {list(w.shape)}.")
    if win_length < n_fft:
        left = (n_fft - win_length) // 2
        w = torch.nn.functional.pad(w, [left, n_fft - win_length - left])
    return w


def stft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, pad_mode="reflect", normalized=False,
         onesided=True, name=None):
    """[seq] or [batch, seq] -> [(batch,) n_fft//2+1 (onesided) or n_fft, num_frames] complex."""
    t = T(x)
    if t.dim() not in (1, 2):
        raise ValueError(f"x should be a 1D or 2D real tensor, but got rank of x is {t.dim()}")
    squeeze = t.dim() == 1
    if squeeze:
        t = t.unsqueeze(0)
    hop_length = n_fft // 4 if hop_length is None else hop_length
    win_length = n_fft if win_length is None else win_length
    if hop_length <= 0:
        raise ValueError(f"hop_length should be > 0, but got {hop_length}.")
    if not 0 < win_length <= n_fft:
        raise ValueError(f"win_length should be in (0, n_fft({n_fft})], but got {win_length}.")
    w = _padded_window(window, win_length, n_fft, t.dtype if not t.is_complex() else torch.float32, t.device)
    if center:
        if pad_mode not in ("constant", "reflect"):
            raise ValueError(f'pad_mode should be "reflect" or "constant", but got "{pad_mode}".')
        p = n_fft // 2
        t = torch.nn.functional.pad(t.unsqueeze(1), [p, p], mode=pad_mode).squeeze(1)
    if not 0 < n_fft <= t.shape[-1]:
        raise ValueError(f"n_fft should be in (0, seq_length({t.shape[-1]})], but got {n_fft}.")
    frames = T(frame(_wrap(t), n_fft, hop_length, axis=-1)).transpose(1, 2)  # [batch, n_frames, n_fft]
    frames = frames * w
    norm = "ortho" if normalized else "backward"
    if frames.is_complex() or w.is_complex():
        if onesided:
            raise ValueError("onesided should be False when input or window is a complex Tensor.")
        out = _fft._c2c(frames, [2], norm, True)
    else:
        out = _fft._r2c(frames, [2], norm, True, onesided)
    out = out.transpose(1, 2)                                        # [batch, freq, n_frames]
    return _wrap(out.squeeze(0) if squeeze else out)


def istft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, normalized=False, onesided=True,
          length=None, return_complex=False, name=None):
    """Inverse of stft by weighted overlap-add: sum_f w * ifft(X_f) / sum_f w^2 (the window must satisfy the
    nonzero overlap-add constraint)."""
    t = T(x)
    if not t.is_complex():
        raise TypeError("istft expects a complex64 / complex128 input")
    if t.dim() not in (2, 3):
        raise ValueError(f"x should be a 2D or 3D complex tensor, but got rank of x is {t.dim()}")
    squeeze = t.dim() == 2
    if squeeze:
        t = t.unsqueeze(0)
    hop_length = n_fft // 4 if hop_length is None else hop_length
    win_length = n_fft if win_length is None else win_length
    if not 0 < hop_length <= win_length:
        raise ValueError(f"hop_length should be in (0, win_length({win_length})], but got {hop_length}.")
    if not 0 < win_length <= n_fft:
        raise ValueError(f"win_length should be in (0, n_fft({n_fft})], but got {win_length}.")
    n_frames, fft_size = t.shape[-1], t.shape[-2]
    if onesided and fft_size != n_fft // 2 + 1:
        raise ValueError(f"fft_size should be equal to n_fft // 2 + 1({n_fft // 2 + 1}) when onesided is True, "
                         f"but got {fft_size}.")
    if not onesided and fft_size != n_fft:
        raise ValueError(f"fft_size should be equal to n_fft({n_fft}) when onesided is False, but got {fft_size}.")
    real_dt = torch.float64 if t.dtype == torch.complex128 else torch.float32
    w = _padded_window(window, win_length, n_fft, real_dt, t.device)
    spec = t.transpose(1, 2)                                         # [batch, n_frames, freq]
    norm = "ortho" if normalized else "backward"
    if return_complex:
        if onesided:
            raise ValueError("onesided should be False when input(output of istft) or window is a complex Tensor.")
        frames = _fft._c2c(spec, [2], norm, False)
    else:
        if w.is_complex():
            raise ValueError("Data type of window should not be complex when return_complex is False.")
        if onesided:
            frames = _fft._c2r(spec, [2], norm, False, n_fft)
        else:
            frames = _fft._c2r(spec[..., :n_fft // 2 + 1], [2], norm, False, n_fft)
    frames = frames * w                                              # [batch, n_frames, n_fft]
    sig = T(overlap_add(_wrap(frames.transpose(1, 2)), hop_length, axis=-1))          # [batch, seq]
    env = T(overlap_add(_wrap((w * w.conj() if w.is_complex() else w * w).reshape(n_fft, 1).expand(n_fft, n_frames)),
                        hop_length, axis=-1))
    start = n_fft // 2 if center else 0
    if length is None:
        end = sig.shape[-1] - (n_fft // 2 if center else 0)
    else:
        end = start + length
    sig = sig[..., start:end]
    env = env[start:end]
    if bool((env.abs() < 1e-11).any()):
        raise ValueError("Abort istft because Nonzero Overlap Add (NOLA) condition failed. For more information "
                         "about NOLA constraint please see `scipy.signal.check_NOLA`.")
    sig = sig / env
    if length is not None and sig.shape[-1] < length:
        sig = torch.nn.functional.pad(sig, [0, length - sig.shape[-1]])
    return _wrap(sig.squeeze(0) if squeeze else sig)


__all__ = ["stft", "istft"]
