"""paddle.signal. Reference: python/paddle/signal.py."""
from __future__ import annotations

import torch

from .framework.tensor import _wrap
from .tensor._helpers import T


def stft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, pad_mode="reflect", normalized=False,
         onesided=True, name=None):
    return _wrap(torch.stft(T(x), n_fft, hop_length, win_length, T(window), center, pad_mode, normalized, onesided,
                            return_complex=True))


def istft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, normalized=False, onesided=True,
          length=None, return_complex=False, name=None):
    return _wrap(torch.istft(T(x), n_fft, hop_length, win_length, T(window), center, normalized, onesided, length,
                             return_complex))
