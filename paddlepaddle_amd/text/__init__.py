"""paddle.text: viterbi decoding + dataset readers. Reference: python/paddle/text/ (viterbi_decode.py
ViterbiDecoder / viterbi_decode; datasets/: Imdb, Imikolov, Movielens, UCIHousing, WMT14, WMT16, Conll05).
Datasets read local copies only (no network)."""
from __future__ import annotations

import os
import tarfile

import numpy as np
import torch

from .. import nn
from ..framework.tensor import Tensor, _wrap
from ..io import Dataset


def viterbi_decode(potentials, transition_params, lengths, include_bos_eos_tag=True, name=None):
    """potentials [B, T, N], transitions [N, N], lengths [B] -> (scores [B], paths [B, T])."""
    emit = potentials._t.float()
    trans = transition_params._t.float()
    lens = lengths._t.long()
    B, T, N = emit.shape
    if include_bos_eos_tag:
        # tags N-2 = BOS, N-1 = EOS (reference convention)
        start = trans[N - 2].clone()
        stop = trans[:, N - 1].clone()
    else:
        start = torch.zeros(N, device=emit.device)
        stop = torch.zeros(N, device=emit.device)
    alpha = emit[:, 0] + start
    back = []
    for t in range(1, T):
        score = alpha[:, :, None] + trans[None]  # [B, from, to]
        best, arg = score.max(1)
        new = best + emit[:, t]
        active = (t < lens)[:, None]
        alpha = torch.where(active, new, alpha)
        back.append(torch.where(active, arg, torch.arange(N, device=emit.device).expand(B, N)))
    alpha = alpha + stop
    scores, last = alpha.max(-1)
    path = [last]
    for bp in reversed(back):
        last = bp.gather(1, last[:, None])[:, 0]
        path.append(last)
    path = torch.stack(path[::-1], 1)
    # positions beyond each length are padding: zero them
    mask = torch.arange(T, device=emit.device)[None] < lens[:, None]
    return _wrap(scores), _wrap(torch.where(mask, path, torch.zeros_like(path)))


class ViterbiDecoder(nn.Layer):
    def __init__(self, transitions, include_bos_eos_tag=True, name=None):
        super().__init__()
        self.transitions = transitions
        self.include_bos_eos_tag = include_bos_eos_tag

    def forward(self, potentials, lengths):
        return viterbi_decode(potentials, self.transitions, lengths, self.include_bos_eos_tag)


def _need(p, what):
    if p is None or not os.path.exists(p):
        raise FileNotFoundError(f"{what}: local file {p!r} not found (no network; downloads are disabled)")


class UCIHousing(Dataset):
    """whitespace-separated 14-column housing data file."""

    def __init__(self, data_file=None, mode="train", download=False):
        _need(data_file, "UCIHousing")
        data = np.loadtxt(data_file).astype("float32").reshape(-1, 14)
        mx, mn, avg = data.max(0), data.min(0), data.mean(0)
        feats = (data[:, :13] - avg[:13]) / (mx[:13] - mn[:13])
        data = np.concatenate([feats, data[:, 13:]], 1)
        cut = int(len(data) * 0.8)
        self.data = data[:cut] if mode == "train" else data[cut:]

    def __getitem__(self, idx):
        d = self.data[idx]
        return d[:-1], d[-1:]

    def __len__(self):
        return len(self.data)


class Imdb(Dataset):
    """aclImdb tarball: reviews tokenised on whitespace/punctuation, word dict built from train."""

    def __init__(self, data_file=None, mode="train", cutoff=150, download=False):
        _need(data_file, "Imdb")
        import re
        self.docs, self.labels = [], []
        pat = re.compile(rf"aclImdb/{mode}/(pos|neg)/.*\.txt$")
        freq = {}
        raw = []
        with tarfile.open(data_file) as tf:
            for m in tf.getmembers():
                g = pat.match(m.name)
                if g:
                    words = re.sub(r"[^\w\s]", " ", tf.extractfile(m).read().decode("utf-8", "ignore").lower()).split()
                    raw.append((words, 0 if g.group(1) == "pos" else 1))
                    for w in words:
                        freq[w] = freq.get(w, 0) + 1
        vocab = sorted([w for w, c in freq.items() if c > cutoff], key=lambda w: (-freq[w], w))
        self.word_idx = {w: i for i, w in enumerate(vocab)}
        unk = len(self.word_idx)
        self.word_idx["<unk>"] = unk
        for words, lab in raw:
            self.docs.append(np.array([self.word_idx.get(w, unk) for w in words], dtype="int64"))
            self.labels.append(np.array([lab], dtype="int64"))

    def __getitem__(self, idx):
        return self.docs[idx], self.labels[idx]

    def __len__(self):
        return len(self.docs)


class Imikolov(Dataset):
    def __init__(self, data_file=None, data_type="NGRAM", window_size=-1, mode="train", min_word_freq=50,
                 download=False):
        _need(data_file, "Imikolov")
        name = {"train": "ptb.train.txt", "test": "ptb.valid.txt"}[mode]
        with tarfile.open(data_file) as tf:
            text = [m for m in tf.getmembers() if m.name.endswith(name)]
            lines = tf.extractfile(text[0]).read().decode().splitlines()
        freq = {}
        for l in lines:
            for w in l.split():
                freq[w] = freq.get(w, 0) + 1
        vocab = sorted([w for w, c in freq.items() if c >= min_word_freq], key=lambda w: (-freq[w], w))
        self.word_idx = {w: i for i, w in enumerate(vocab)}
        for s in ("<s>", "<e>", "<unk>"):
            self.word_idx.setdefault(s, len(self.word_idx))
        unk = self.word_idx["<unk>"]
        self.data = []
        for l in lines:
            ids = [self.word_idx["<s>"]] + [self.word_idx.get(w, unk) for w in l.split()] + [self.word_idx["<e>"]]
            if data_type == "NGRAM":
                for i in range(window_size, len(ids) + 1):
                    self.data.append(tuple(np.array([x]) for x in ids[i - window_size:i]))
            else:
                self.data.append((np.array(ids[:-1]), np.array(ids[1:])))

    def __getitem__(self, idx):
        return self.data[idx]

    def __len__(self):
        return len(self.data)


class _Unavailable(Dataset):
    def __init__(self, *a, data_file=None, **k):
        _need(data_file, type(self).__name__)
        raise NotImplementedError(f"{type(self).__name__}: parser for the local archive format is not provided")


class Movielens(_Unavailable):
    pass


class WMT14(_Unavailable):
    pass


class WMT16(_Unavailable):
    pass


class Conll05st(_Unavailable):
    pass


class datasets:  # paddle.text.datasets namespace
    UCIHousing = UCIHousing
    Imdb = Imdb
    Imikolov = Imikolov
    Movielens = Movielens
    WMT14 = WMT14
    WMT16 = WMT16
    Conll05st = Conll05st
