"""paddle.metric. Reference: python/paddle/metric/metrics.py (Metric, Accuracy, Precision, Recall,
Auc, accuracy). ``compute`` runs on the device (top-k on the logits where they live); ``update``
accumulates on the host in numpy, as in the reference."""
from __future__ import annotations

import abc

import numpy as np
import torch

from ..framework.tensor import Tensor, _wrap


def _np(x):
    if isinstance(x, Tensor):
        return x.numpy()
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class Metric(abc.ABC):
    def __init__(self):
        pass

    @abc.abstractmethod
    def reset(self):
        ...

    @abc.abstractmethod
    def update(self, *args):
        ...

    @abc.abstractmethod
    def accumulate(self):
        ...

    @abc.abstractmethod
    def name(self):
        ...

    def compute(self, *args):
        return args


class Accuracy(Metric):
    def __init__(self, topk=(1,), name=None, *args, **kwargs):
        super().__init__()
        self.topk = topk
        self.maxk = max(topk)
        self._init_name(name)
        self.reset()

    def compute(self, pred, label, *args):
        p = pred._t if isinstance(pred, Tensor) else torch.as_tensor(pred)
        lb = label._t if isinstance(label, Tensor) else torch.as_tensor(label)
        idx = p.topk(self.maxk, dim=-1).indices
        if lb.dim() == p.dim() and lb.shape[-1] != 1:  # one-hot / soft labels
            lb = lb.argmax(-1, keepdim=True)
        elif lb.dim() == p.dim() - 1:
            lb = lb.unsqueeze(-1)
        correct = (idx == lb.to(idx.dtype)).to(torch.float32)
        return _wrap(correct)

    def update(self, correct, *args):
        c = _np(correct)
        num = c.shape[0] if c.ndim else 1
        accs = []
        for i, k in enumerate(self.topk):
            ck = c[..., :k].sum()
            accs.append(float(ck) / max(num, 1))
            self.total[i] += ck
            self.count[i] += num
        return accs[0] if len(self.topk) == 1 else accs

    def reset(self):
        self.total = [0.0] * len(self.topk)
        self.count = [0] * len(self.topk)

    def accumulate(self):
        res = [float(t) / c if c > 0 else 0.0 for t, c in zip(self.total, self.count)]
        return res[0] if len(self.topk) == 1 else res

    def _init_name(self, name):
        name = name or "acc"
        self._name = [f"{name}_top{k}" for k in self.topk] if self.maxk != 1 else [name]

    def name(self):
        return self._name


class Precision(Metric):
    def __init__(self, name="precision", *args, **kwargs):
        super().__init__()
        self.tp = 0
        self.fp = 0
        self._name = name

    def update(self, preds, labels):
        p = np.rint(_np(preds)).astype("int32").reshape(-1)
        lb = _np(labels).astype("int32").reshape(-1)
        self.tp += int(((p == 1) & (lb == 1)).sum())
        self.fp += int(((p == 1) & (lb == 0)).sum())

    def reset(self):
        self.tp = 0
        self.fp = 0

    def accumulate(self):
        ap = self.tp + self.fp
        return float(self.tp) / ap if ap != 0 else 0.0

    def name(self):
        return self._name


class Recall(Metric):
    def __init__(self, name="recall", *args, **kwargs):
        super().__init__()
        self.tp = 0
        self.fn = 0
        self._name = name

    def update(self, preds, labels):
        p = np.rint(_np(preds)).astype("int32").reshape(-1)
        lb = _np(labels).astype("int32").reshape(-1)
        self.tp += int(((p == 1) & (lb == 1)).sum())
        self.fn += int(((p == 0) & (lb == 1)).sum())

    def accumulate(self):
        r = self.tp + self.fn
        return float(self.tp) / r if r != 0 else 0.0

    def reset(self):
        self.tp = 0
        self.fn = 0

    def name(self):
        return self._name


class Auc(Metric):
    """Histogram (bucketed threshold) ROC / PR AUC, like the reference."""

    def __init__(self, curve="ROC", num_thresholds=4095, name="auc", *args, **kwargs):
        super().__init__()
        self._curve = curve
        self._num_thresholds = num_thresholds
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = _np(preds)
        lb = _np(labels).reshape(-1)
        pos = p[:, 1] if p.ndim == 2 else p.reshape(-1)
        bins = np.clip((pos * self._num_thresholds).astype("int64"), 0, self._num_thresholds)
        np.add.at(self._stat_pos, bins[lb != 0], 1)
        np.add.at(self._stat_neg, bins[lb == 0], 1)

    def accumulate(self):
        tot_pos = tot_neg = 0.0
        auc = 0.0
        if self._curve == "PR":
            tp = np.cumsum(self._stat_pos[::-1])
            fp = np.cumsum(self._stat_neg[::-1])
            prec = tp / np.maximum(tp + fp, 1)
            rec = tp / max(tp[-1], 1)
            return float(np.trapz(prec, rec)) if tp[-1] > 0 else 0.0
        for i in range(self._num_thresholds, -1, -1):
            np_, nn_ = tot_pos, tot_neg
            tot_pos += self._stat_pos[i]
            tot_neg += self._stat_neg[i]
            auc += (tot_neg - nn_) * (tot_pos + np_) / 2.0
        return auc / tot_pos / tot_neg if tot_pos > 0 and tot_neg > 0 else 0.0

    def reset(self):
        self._stat_pos = np.zeros(self._num_thresholds + 1, dtype="int64")
        self._stat_neg = np.zeros(self._num_thresholds + 1, dtype="int64")

    def name(self):
        return self._name


def accuracy(input, label, k=1, correct=None, total=None, name=None):
    """Top-k accuracy of a batch as a scalar tensor (reference: metric/metrics.py accuracy)."""
    p = input._t
    lb = label._t
    if lb.dim() == p.dim():
        lb = lb.squeeze(-1)
    idx = p.topk(k, dim=-1).indices
    hit = (idx == lb.unsqueeze(-1).to(idx.dtype)).any(-1).to(torch.float32)
    n = hit.numel()
    c = hit.sum()
    if correct is not None:
        correct._t.copy_(c.to(correct._t.dtype))
    if total is not None:
        total._t.fill_(n)
    return _wrap(c / max(n, 1))
