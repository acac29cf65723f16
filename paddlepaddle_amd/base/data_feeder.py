"""paddle.base.DataFeeder (reference: python/paddle/base/data_feeder.py DataFeeder): converts a mini-batch of
samples (one tuple per sample, one entry per feed variable) into the feed dict of ``Executor.run``."""
from __future__ import annotations

import numpy as np

from ..framework import dtype as _dt


class DataFeeder:
    def __init__(self, feed_list, place=None, program=None):
        self.feed_names, self.feed_shapes, self.feed_dtypes = [], [], []
        for v in feed_list:
            name = v if isinstance(v, str) else (getattr(v, "_name", None) or getattr(v, "name", None))
            if name is None:
                raise TypeError(f"DataFeeder: feed variable {v!r} has no name")
            self.feed_names.append(name)
            self.feed_shapes.append(None if isinstance(v, str) else list(v.shape))
            self.feed_dtypes.append(None if isinstance(v, str) else _dt.convert_dtype(v.dtype))
        self.place = place

    def _column(self, values, shape, dtype):
        arr = np.asarray(values)
        if dtype is not None:
            import torch
            arr = arr.astype(torch.empty((), dtype=_dt.to_torch_dtype(dtype)).numpy().dtype)
        if shape is not None:
            tail = [int(s) for s in shape[1:]]
            if all(s > 0 for s in tail):
                arr = arr.reshape([len(values)] + tail)
        return arr

    def feed(self, iterable):
        samples = list(iterable)
        cols = list(zip(*samples)) if samples else [[] for _ in self.feed_names]
        if len(cols) != len(self.feed_names):
            raise ValueError(f"DataFeeder: each sample has {len(cols)} fields for {len(self.feed_names)} feeds")
        return {n: self._column(list(c), s, d)
                for n, c, s, d in zip(self.feed_names, cols, self.feed_shapes, self.feed_dtypes)}

    def feed_parallel(self, iterable, num_places=None):
        for batch in iterable:
            yield self.feed(batch)

    def decorate_reader(self, reader, multi_devices=False, num_places=None, drop_last=True):
        def gen():
            for batch in reader():
                yield self.feed(batch)
        return gen
