"""paddle.audio: feature extraction (Spectrogram / MelSpectrogram / LogMelSpectrogram / MFCC), window
functions, mel / dct helpers, wav IO. Reference: python/paddle/audio/ (features/layers.py,
functional/functional.py, functional/window.py, backends/wave_backend.py).
STFT runs on the device FFT (``paddle.signal.stft``)."""
from __future__ import annotations

import math
import wave

import numpy as np
import torch

from .. import nn
from ..framework.tensor import Tensor, _wrap


class functional:
    @staticmethod
    def hz_to_mel(freq, htk=False):
        f = freq._t if isinstance(freq, Tensor) else torch.as_tensor(freq, dtype=torch.float64)
        if htk:
            out = 2595.0 * torch.log10(1.0 + f / 700.0)
        else:
            f_sp = 200.0 / 3
            mels = f / f_sp
            min_log_hz = 1000.0
            min_log_mel = min_log_hz / f_sp
            logstep = math.log(6.4) / 27.0
            out = torch.where(f >= min_log_hz, min_log_mel + torch.log(f.clamp_min(1e-10) / min_log_hz) / logstep, mels)
        return _wrap(out) if isinstance(freq, Tensor) else (float(out) if out.dim() == 0 else out.numpy())

    @staticmethod
    def mel_to_hz(mel, htk=False):
        m = mel._t if isinstance(mel, Tensor) else torch.as_tensor(mel, dtype=torch.float64)
        if htk:
            out = 700.0 * (10.0 ** (m / 2595.0) - 1.0)
        else:
            f_sp = 200.0 / 3
            freqs = f_sp * m
            min_log_hz = 1000.0
            min_log_mel = min_log_hz / f_sp
            logstep = math.log(6.4) / 27.0
            out = torch.where(m >= min_log_mel, min_log_hz * torch.exp(logstep * (m - min_log_mel)), freqs)
        return _wrap(out) if isinstance(mel, Tensor) else (float(out) if out.dim() == 0 else out.numpy())

    @staticmethod
    def mel_frequencies(n_mels=64, f_min=0.0, f_max=11025.0, htk=False, dtype="float32"):
        lo = functional.hz_to_mel(f_min, htk)
        hi = functional.hz_to_mel(f_max, htk)
        mels = torch.linspace(float(lo), float(hi), n_mels, dtype=torch.float64)
        return _wrap(torch.as_tensor(functional.mel_to_hz(mels.numpy(), htk)).float())

    @staticmethod
    def fft_frequencies(sr, n_fft, dtype="float32"):
        return _wrap(torch.linspace(0, sr / 2, 1 + n_fft // 2))

    @staticmethod
    def compute_fbank_matrix(sr, n_fft, n_mels=64, f_min=0.0, f_max=None, htk=False, norm="slaney",
                             dtype="float32"):
        f_max = f_max or sr / 2
        fftfreqs = functional.fft_frequencies(sr, n_fft)._t.double()
        mel_f = functional.mel_frequencies(n_mels + 2, f_min, f_max, htk)._t.double()
        fdiff = mel_f[1:] - mel_f[:-1]
        ramps = mel_f[:, None] - fftfreqs[None]
        lower = -ramps[:-2] / fdiff[:-1, None]
        upper = ramps[2:] / fdiff[1:, None]
        w = torch.clamp(torch.minimum(lower, upper), min=0)
        if norm == "slaney":
            enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
            w = w * enorm[:, None]
        return _wrap(w.float())

    @staticmethod
    def power_to_db(spect, ref_value=1.0, amin=1e-10, top_db=80.0):
        s = spect._t
        db = 10.0 * torch.log10(s.clamp_min(amin)) - 10.0 * math.log10(max(ref_value, amin))
        if top_db is not None:
            db = torch.maximum(db, db.max() - top_db)
        return _wrap(db)

    @staticmethod
    def create_dct(n_mfcc, n_mels, norm="ortho", dtype="float32"):
        n = torch.arange(n_mels, dtype=torch.float64)
        k = torch.arange(n_mfcc, dtype=torch.float64)[:, None]
        dct = torch.cos(math.pi / n_mels * (n + 0.5) * k)
        if norm == "ortho":
            dct[0] *= 1.0 / math.sqrt(2.0)
            dct *= math.sqrt(2.0 / n_mels)
        else:
            dct *= 2.0
        return _wrap(dct.t().float())

    @staticmethod
    def get_window(window, win_length, fftbins=True, dtype="float64"):
        """Window of ``win_length`` samples; ``fftbins`` -> periodic (the symmetric window of length n + 1
        without its last sample). ``window`` is a name or (name, *params). Reference:
        python/paddle/audio/functional/window.py get_window (same window family and parameter order)."""
        if isinstance(window, (tuple, list)):
            name, params = window[0], tuple(window[1:])
        else:
            name, params = window, ()
        n = int(win_length)
        m = n + 1 if fftbins else n
        if name not in _WINDOWS:
            raise ValueError(f"Unknown window type: {name}")
        fn, needs = _WINDOWS[name]
        if len(params) < needs:
            raise ValueError(f"The '{name}' window needs one or more parameters -- pass a tuple.")
        w = fn(m, *params) if m > 1 else torch.ones(m, dtype=torch.float64)
        w = w[:n]
        from ..framework import dtype as _dtm
        return _wrap(w.to(_dtm.to_torch_dtype(dtype)))


def _cos_sum(m, coeffs):
    x = torch.linspace(-math.pi, math.pi, m, dtype=torch.float64)
    w = torch.zeros(m, dtype=torch.float64)
    for k, a in enumerate(coeffs):
        w = w + a * torch.cos(k * x)
    return w


def _w_general_gaussian(m, p, sig):
    n = torch.arange(m, dtype=torch.float64) - (m - 1.0) / 2.0
    return torch.exp(-0.5 * torch.abs(n / sig) ** (2 * p))


def _w_exponential(m, center=None, tau=1.0):
    c = (m - 1) / 2 if center is None else center
    return torch.exp(-torch.abs(torch.arange(m, dtype=torch.float64) - c) / tau)


def _w_triang(m):
    n = torch.arange(1, (m + 1) // 2 + 1, dtype=torch.float64)
    w = 2 * n / (m + 1.0) if m % 2 == 1 else (2 * n - 1.0) / m
    return torch.cat([w, w.flip(0)[1:]]) if m % 2 == 1 else torch.cat([w, w.flip(0)])


def _w_bohman(m):
    fac = torch.abs(torch.linspace(-1, 1, m, dtype=torch.float64)[1:-1])
    w = (1 - fac) * torch.cos(math.pi * fac) + 1.0 / math.pi * torch.sin(math.pi * fac)
    z = torch.zeros(1, dtype=torch.float64)
    return torch.cat([z, w, z])


def _w_tukey(m, alpha=0.5):
    if alpha <= 0:
        return torch.ones(m, dtype=torch.float64)
    if alpha >= 1:
        return _cos_sum(m, [0.5, 0.5])
    n = torch.arange(m, dtype=torch.float64)
    width = math.floor(alpha * (m - 1) / 2.0)
    w = torch.ones(m, dtype=torch.float64)
    n1, n3 = n[:width + 1], n[m - width - 1:]
    w[:width + 1] = 0.5 * (1 + torch.cos(math.pi * (-1 + 2.0 * n1 / alpha / (m - 1))))
    w[m - width - 1:] = 0.5 * (1 + torch.cos(math.pi * (-2.0 / alpha + 1 + 2.0 * n3 / alpha / (m - 1))))
    return w


def _w_taylor(m, nbar=4, sll=30, norm=True):
    b = 10 ** (sll / 20)
    a = math.acosh(b) / math.pi
    s2 = nbar ** 2 / (a ** 2 + (nbar - 0.5) ** 2)
    ma = torch.arange(1, nbar, dtype=torch.float64)
    fm = torch.empty(nbar - 1, dtype=torch.float64)
    signs = torch.empty_like(ma)
    signs[::2] = 1
    signs[1::2] = -1
    m2 = ma * ma
    for mi in range(len(ma)):
        numer = signs[mi] * torch.prod(1 - m2[mi] / s2 / (a ** 2 + (ma - 0.5) ** 2))
        denom = 2 * torch.prod(1 - m2[mi] / torch.cat([m2[:mi], m2[mi + 1:]]))
        fm[mi] = numer / denom
    x = torch.arange(m, dtype=torch.float64)

    def w_of(xx):
        return 1 + 2 * torch.matmul(fm, torch.cos(2 * math.pi * ma.unsqueeze(1) * (xx - m / 2.0 + 0.5) / m))
    w = w_of(x)
    if norm:
        w = w / w_of(torch.tensor([(m - 1) / 2.0], dtype=torch.float64))
    return w


def _w_kaiser(m, beta=12.0):
    n = torch.arange(m, dtype=torch.float64)
    alpha = (m - 1) / 2.0
    return torch.special.i0(beta * torch.sqrt(1 - ((n - alpha) / alpha) ** 2)) / torch.special.i0(
        torch.tensor(float(beta), dtype=torch.float64))


def _w_gaussian(m, std):
    n = torch.arange(m, dtype=torch.float64) - (m - 1.0) / 2.0
    return torch.exp(-n ** 2 / (2 * std * std))


def _w_bartlett(m):
    n = torch.arange(m, dtype=torch.float64)
    return torch.where(n <= (m - 1) / 2.0, 2.0 * n / (m - 1), 2.0 - 2.0 * n / (m - 1))


_WINDOWS = {
    "hamming": (lambda m: _cos_sum(m, [0.54, 0.46]), 0),
    "hann": (lambda m: _cos_sum(m, [0.5, 0.5]), 0),
    "blackman": (lambda m: _cos_sum(m, [0.42, 0.50, 0.08]), 0),
    "nuttall": (lambda m: _cos_sum(m, [0.3635819, 0.4891775, 0.1365995, 0.0106411]), 0),
    "cosine": (lambda m: torch.sin(math.pi / m * (torch.arange(m, dtype=torch.float64) + 0.5)), 0),
    "gaussian": (_w_gaussian, 1),
    "general_gaussian": (_w_general_gaussian, 2),
    "exponential": (_w_exponential, 0),
    "triang": (_w_triang, 0),
    "bohman": (_w_bohman, 0),
    "tukey": (_w_tukey, 0),
    "taylor": (_w_taylor, 0),
    "bartlett": (_w_bartlett, 0),
    "kaiser": (_w_kaiser, 0),
    "boxcar": (lambda m: torch.ones(m, dtype=torch.float64), 0),
    "rect": (lambda m: torch.ones(m, dtype=torch.float64), 0),
    "rectangular": (lambda m: torch.ones(m, dtype=torch.float64), 0),
}


class Spectrogram(nn.Layer):
    def __init__(self, n_fft=512, hop_length=512, win_length=None, window="hann", power=1.0, center=True,
                 pad_mode="reflect", dtype="float32"):  # reference audio/features/layers.py defaults
        super().__init__()
        self.n_fft, self.hop = n_fft, hop_length or (win_length or n_fft) // 4
        self.win_length = win_length or n_fft
        self.power, self.center, self.pad_mode = power, center, pad_mode
        self.register_buffer("window", functional.get_window(window, self.win_length, dtype=dtype))

    def forward(self, x):
        t = x._t
        spec = torch.stft(t, self.n_fft, self.hop, self.win_length, self.window._t.to(t.device, t.dtype),
                          center=self.center, pad_mode=self.pad_mode, return_complex=True)
        return _wrap(spec.abs() ** self.power)


class MelSpectrogram(nn.Layer):
    def __init__(self, sr=22050, n_fft=2048, hop_length=512, win_length=None, window="hann", power=2.0, center=True,
                 pad_mode="reflect", n_mels=64, f_min=50.0, f_max=None, htk=False, norm="slaney", dtype="float32"):
        super().__init__()
        self._spec = Spectrogram(n_fft, hop_length, win_length, window, power, center, pad_mode, dtype)
        self.register_buffer("fbank_matrix", functional.compute_fbank_matrix(sr, n_fft, n_mels, f_min, f_max, htk,
                                                                             norm))

    def forward(self, x):
        s = self._spec(x)._t
        return _wrap(torch.matmul(self.fbank_matrix._t.to(s.device, s.dtype), s))


class LogMelSpectrogram(nn.Layer):
    def __init__(self, sr=22050, n_fft=512, hop_length=None, win_length=None, window="hann", power=2.0, center=True,
                 pad_mode="reflect", n_mels=64, f_min=50.0, f_max=None, htk=False, norm="slaney", ref_value=1.0,
                 amin=1e-10, top_db=None, dtype="float32"):
        super().__init__()
        self._mel = MelSpectrogram(sr, n_fft, hop_length, win_length, window, power, center, pad_mode, n_mels, f_min,
                                   f_max, htk, norm, dtype)
        self.ref_value, self.amin, self.top_db = ref_value, amin, top_db

    def forward(self, x):
        return functional.power_to_db(self._mel(x), self.ref_value, self.amin, self.top_db)


class MFCC(nn.Layer):
    def __init__(self, sr=22050, n_mfcc=40, n_fft=512, hop_length=None, win_length=None, window="hann", power=2.0,
                 center=True, pad_mode="reflect", n_mels=64, f_min=50.0, f_max=None, htk=False, norm="slaney",
                 ref_value=1.0, amin=1e-10, top_db=None, dtype="float32"):
        super().__init__()
        self._log_mel = LogMelSpectrogram(sr, n_fft, hop_length, win_length, window, power, center, pad_mode, n_mels,
                                          f_min, f_max, htk, norm, ref_value, amin, top_db, dtype)
        self.register_buffer("dct_matrix", functional.create_dct(n_mfcc, n_mels))

    def forward(self, x):
        lm = self._log_mel(x)._t  # [B, n_mels, frames]
        return _wrap(torch.matmul(lm.transpose(-1, -2), self.dct_matrix._t.to(lm.device, lm.dtype)).transpose(-1, -2))


class features:
    Spectrogram = Spectrogram
    MelSpectrogram = MelSpectrogram
    LogMelSpectrogram = LogMelSpectrogram
    MFCC = MFCC


def load(filepath, frame_offset=0, num_frames=-1, normalize=True, channels_first=True):
    with wave.open(filepath, "rb") as w:
        sr, nch, width = w.getframerate(), w.getnchannels(), w.getsampwidth()
        w.setpos(frame_offset)
        raw = w.readframes(w.getnframes() - frame_offset if num_frames < 0 else num_frames)
    dt = {1: np.uint8, 2: np.int16, 4: np.int32}[width]
    a = np.frombuffer(raw, dtype=dt).reshape(-1, nch).astype("float32")
    if normalize:
        a = (a - 128) / 128.0 if width == 1 else a / float(2 ** (8 * width - 1))
    t = torch.from_numpy(a.T.copy() if channels_first else a.copy())
    return _wrap(t), sr


def save(filepath, src, sample_rate, channels_first=True, encoding=None, bits_per_sample=16):
    a = src.numpy() if isinstance(src, Tensor) else np.asarray(src)
    if channels_first:
        a = a.T
    a = np.clip(a, -1, 1)
    pcm = (a * (2 ** (bits_per_sample - 1) - 1)).astype(np.int16 if bits_per_sample == 16 else np.int32)
    with wave.open(filepath, "wb") as w:
        w.setnchannels(pcm.shape[1] if pcm.ndim == 2 else 1)
        w.setsampwidth(bits_per_sample // 8)
        w.setframerate(sample_rate)
        w.writeframes(pcm.tobytes())


def info(filepath):
    with wave.open(filepath, "rb") as w:
        return {"sample_rate": w.getframerate(), "num_frames": w.getnframes(), "num_channels": w.getnchannels(),
                "bits_per_sample": 8 * w.getsampwidth()}


class backends:
    @staticmethod
    def list_available_backends():
        return ["wave_backend"]

    @staticmethod
    def get_current_backend():
        return "wave_backend"

    @staticmethod
    def set_backend(name):
        if name != "wave_backend":
            raise ValueError("only the built-in wave backend is available")


class _AudioDataset:
    """Local-file audio classification dataset (no download: point ``data_dir`` at an extracted copy).
    Returns (waveform or feature, label) pairs; feat_type 'raw' | 'melspectrogram' | 'mfcc' | ...
    (reference python/paddle/audio/datasets/{esc50,tess}.py)."""
    n_class = 0

    def __init__(self, mode="train", split=1, feat_type="raw", archive=None, data_dir=None, **kwargs):
        import os
        if data_dir is None or not os.path.isdir(data_dir):
            raise RuntimeError(f"{type(self).__name__}: no network access — pass data_dir= pointing at the "
                               "extracted dataset")
        self.mode, self.split, self.feat_type, self.kwargs = mode, split, feat_type, kwargs
        self.files, self.labels = self._scan(data_dir)

    def _scan(self, data_dir):
        raise NotImplementedError

    def __len__(self):
        return len(self.files)

    def __getitem__(self, idx):
        wav, sr = load(self.files[idx])
        x = wav
        if self.feat_type != "raw":
            layer = {"melspectrogram": MelSpectrogram, "logmelspectrogram": LogMelSpectrogram,
                     "mfcc": MFCC, "spectrogram": Spectrogram}[self.feat_type.lower()]
            x = layer(sr=sr, **self.kwargs) if layer is not Spectrogram else layer(**self.kwargs)
            x = x(wav)
        return x, self.labels[idx]


class ESC50(_AudioDataset):
    n_class = 50

    def _scan(self, data_dir):
        import csv
        import os
        meta = os.path.join(data_dir, "meta", "esc50.csv")
        files, labels = [], []
        with open(meta) as f:
            for row in csv.DictReader(f):
                fold = int(row["fold"])
                if (self.mode == "train") == (fold != self.split):
                    files.append(os.path.join(data_dir, "audio", row["filename"]))
                    labels.append(int(row["target"]))
        return files, labels


class TESS(_AudioDataset):
    n_class = 7
    label_list = ["angry", "disgust", "fear", "happy", "neutral", "ps", "sad"]

    def _scan(self, data_dir):
        import os
        files, labels = [], []
        for root, _, names in os.walk(data_dir):
            for i, n in enumerate(sorted(names)):
                if not n.endswith(".wav"):
                    continue
                emo = n.rsplit(".", 1)[0].split("_")[-1].lower()
                if emo not in self.label_list:
                    continue
                if (self.mode == "train") == (i % 5 != self.split - 1):
                    files.append(os.path.join(root, n))
                    labels.append(self.label_list.index(emo))
        return files, labels


class datasets:  # namespace: paddle.audio.datasets.ESC50 / TESS
    ESC50 = ESC50
    TESS = TESS


import sys as _sys  # noqa: E402
for _n in ("functional", "features", "backends", "datasets"):
    _sys.modules[__name__ + "." + _n] = globals()[_n]
