"""paddle.io — datasets, samplers, DataLoader.
Reference: python/paddle/io/reader.py:262 (DataLoader), python/paddle/io/dataloader/*.

Design: the worker pool (multiprocess, shared-memory transport) is the PyTorch-ROCm one; batch
assembly of numpy samples into contiguous host buffers is done by the native C++ collator
(``csrc/runtime`` → ``_C_runtime``). With ``use_buffer_reader`` on a GPU the loader double-buffers:
the next batch is staged into the native pinned pool (``csrc/runtime/pinned_pool.cpp``) and copied
on a side HIP stream while the caller computes on the current one.
"""
from __future__ import annotations

import bisect
import math
import numbers

import numpy as np
import torch
import torch.utils.data as _tud

from ..framework.tensor import Tensor, _wrap
from ..framework.place import _get_torch_device


class Dataset:
    def __getitem__(self, idx):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError


class IterableDataset(Dataset):
    def __iter__(self):
        raise NotImplementedError


class TensorDataset(Dataset):
    def __init__(self, tensors):
        self.tensors = tensors
        n = tensors[0].shape[0]
        assert all(t.shape[0] == n for t in tensors)

    def __getitem__(self, idx):
        return tuple(t[idx] for t in self.tensors)

    def __len__(self):
        return self.tensors[0].shape[0]


class ComposeDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __len__(self):
        return len(self.datasets[0])

    def __getitem__(self, idx):
        out = []
        for d in self.datasets:
            s = d[idx]
            out.extend(s if isinstance(s, (list, tuple)) else [s])
        return tuple(out)


class ChainDataset(IterableDataset):
    def __init__(self, datasets):
        self.datasets = datasets

    def __iter__(self):
        for d in self.datasets:
            yield from d


class ConcatDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)
        self.cumulative_sizes = list(np.cumsum([len(d) for d in self.datasets]))

    def __len__(self):
        return self.cumulative_sizes[-1]

    def __getitem__(self, idx):
        if idx < 0:
            idx += len(self)
        di = bisect.bisect_right(self.cumulative_sizes, idx)
        prev = 0 if di == 0 else self.cumulative_sizes[di - 1]
        return self.datasets[di][idx - prev]


class Subset(Dataset):
    def __init__(self, dataset, indices):
        self.dataset, self.indices = dataset, indices

    def __getitem__(self, idx):
        return self.dataset[self.indices[idx]]

    def __len__(self):
        return len(self.indices)


def random_split(dataset, lengths, generator=None):
    n = len(dataset)
    if all(0 <= l <= 1 for l in lengths) and abs(sum(lengths) - 1) < 1e-6 and sum(lengths) != n:
        sizes = [int(math.floor(n * f)) for f in lengths]
        for i in range(n - sum(sizes)):
            sizes[i % len(sizes)] += 1
        lengths = sizes
    perm = np.random.permutation(n).tolist()
    out, off = [], 0
    for l in lengths:
        out.append(Subset(dataset, perm[off:off + l]))
        off += l
    return out


# ---------------------------------------------------------------------------- samplers
class Sampler:
    def __init__(self, data_source=None):
        self.data_source = data_source

    def __iter__(self):
        raise NotImplementedError


class SequenceSampler(Sampler):
    def __iter__(self):
        return iter(range(len(self.data_source)))

    def __len__(self):
        return len(self.data_source)


class RandomSampler(Sampler):
    def __init__(self, data_source, replacement=False, num_samples=None, generator=None):
        super().__init__(data_source)
        self.replacement = replacement
        self._num_samples = num_samples
        self.generator = generator

    @property
    def num_samples(self):
        return len(self.data_source) if self._num_samples is None else self._num_samples

    def __iter__(self):
        n = len(self.data_source)
        if self.replacement:
            return iter(np.random.randint(0, n, self.num_samples).tolist())
        return iter(np.random.permutation(n)[: self.num_samples].tolist())

    def __len__(self):
        return self.num_samples


class WeightedRandomSampler(Sampler):
    def __init__(self, weights, num_samples, replacement=True):
        super().__init__(None)
        self.weights = np.asarray(weights._t.cpu().numpy() if isinstance(weights, Tensor) else weights, np.float64)
        self.num_samples, self.replacement = num_samples, replacement

    def __iter__(self):
        p = self.weights / self.weights.sum()
        return iter(np.random.choice(len(p), self.num_samples, self.replacement, p).tolist())

    def __len__(self):
        return self.num_samples


class SubsetRandomSampler(Sampler):
    def __init__(self, indices, generator=None):
        super().__init__(None)
        self.indices = indices

    def __iter__(self):
        return iter([self.indices[i] for i in np.random.permutation(len(self.indices))])

    def __len__(self):
        return len(self.indices)


class BatchSampler(Sampler):
    def __init__(self, dataset=None, sampler=None, shuffle=False, batch_size=1, drop_last=False):
        super().__init__(dataset)
        if sampler is None:
            sampler = RandomSampler(dataset) if shuffle else SequenceSampler(dataset)
        self.sampler, self.batch_size, self.drop_last = sampler, batch_size, drop_last

    def __iter__(self):
        batch = []
        for i in self.sampler:
            batch.append(i)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if batch and not self.drop_last:
            yield batch

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size


class DistributedBatchSampler(BatchSampler):
    """Shards the (optionally shuffled) index space over data-parallel ranks.
    Reference: python/paddle/io/dataloader/batch_sampler.py DistributedBatchSampler."""

    def __init__(self, dataset, batch_size, num_replicas=None, rank=None, shuffle=False, drop_last=False):
        from ..distributed import collective as C
        self.dataset, self.batch_size, self.shuffle, self.drop_last = dataset, batch_size, shuffle, drop_last
        self.nranks = num_replicas if num_replicas is not None else C.get_world_size()
        self.local_rank = rank if rank is not None else C.get_rank()
        self.epoch = 0
        self.num_samples = int(math.ceil(len(dataset) * 1.0 / self.nranks))
        self.total_size = self.num_samples * self.nranks

    def __iter__(self):
        n = len(self.dataset)
        idx = np.arange(n)
        if self.shuffle:
            rng = np.random.RandomState(self.epoch)
            rng.shuffle(idx)
            self.epoch += 1
        idx = idx.tolist()
        idx += idx[: (self.total_size - len(idx))]
        idx = idx[self.local_rank: self.total_size: self.nranks]
        batch = []
        for i in idx:
            batch.append(i)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if batch and not self.drop_last:
            yield batch

    def __len__(self):
        n = self.num_samples
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def set_epoch(self, epoch):
        self.epoch = epoch


# ---------------------------------------------------------------------------- collate
def _to_np(x):
    if isinstance(x, Tensor):
        return x.numpy()
    return x


def default_collate_fn(batch):
    """Stack a list of samples. numpy arrays are stacked by the native collator when available."""
    s = batch[0]
    if isinstance(s, (np.ndarray, Tensor)) or isinstance(s, torch.Tensor):
        arrs = [b.numpy() if isinstance(b, Tensor) else (b.numpy() if isinstance(b, torch.Tensor) else b)
                for b in batch]
        from ..utils import native
        out = native.stack_arrays(arrs)
        return torch.from_numpy(out)
    if isinstance(s, numbers.Number) or isinstance(s, np.generic):
        return torch.from_numpy(np.asarray(batch))
    if isinstance(s, (str, bytes)):
        return batch
    if isinstance(s, dict):
        return {k: default_collate_fn([b[k] for b in batch]) for k in s}
    if isinstance(s, (list, tuple)):
        return [default_collate_fn(list(f)) for f in zip(*batch)]
    return batch


def default_convert_fn(batch):
    if isinstance(batch, np.ndarray):
        return torch.from_numpy(batch)
    return batch


class _TorchDS(_tud.Dataset):
    def __init__(self, ds):
        self.ds = ds

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, i):
        return _to_np_nested(self.ds[i])


class _TorchIterDS(_tud.IterableDataset):
    def __init__(self, ds):
        self.ds = ds

    def __iter__(self):
        for s in self.ds:
            yield _to_np_nested(s)


def _to_np_nested(s):
    if isinstance(s, Tensor):
        return s.numpy()
    if isinstance(s, (list, tuple)):
        return type(s)(_to_np_nested(v) for v in s)
    if isinstance(s, dict):
        return {k: _to_np_nested(v) for k, v in s.items()}
    return s


class _BS(_tud.Sampler):
    def __init__(self, bs):
        self.bs = bs

    def __iter__(self):
        return iter(self.bs)

    def __len__(self):
        return len(self.bs)


def _stage_batch(x, device, stream, pinned):
    """CPU batch -> pooled pinned memory -> async copy to ``device`` on ``stream``."""
    if isinstance(x, torch.Tensor):
        if x.device.type != "cpu":
            return x.to(device, non_blocking=True)
        src = x if pinned.is_pooled(x) else pinned.pin(x)
        return pinned.copy_to_device(src, device, stream)
    if isinstance(x, (list, tuple)):
        return [_stage_batch(v, device, stream, pinned) for v in x]
    if isinstance(x, dict):
        return {k: _stage_batch(v, device, stream, pinned) for k, v in x.items()}
    return x


def _record_stream(x, stream):
    if isinstance(x, torch.Tensor):
        x.record_stream(stream)
    elif isinstance(x, (list, tuple)):
        for v in x:
            _record_stream(v, stream)
    elif isinstance(x, dict):
        for v in x.values():
            _record_stream(v, stream)


def _wrap_out(x, device, non_blocking):
    if isinstance(x, torch.Tensor):
        if device is not None and device.type == "cuda":
            x = x.to(device, non_blocking=non_blocking)
        return _wrap(x)
    if isinstance(x, (list, tuple)):
        return [_wrap_out(v, device, non_blocking) for v in x]
    if isinstance(x, dict):
        return {k: _wrap_out(v, device, non_blocking) for k, v in x.items()}
    return x


_worker_info = None


def get_worker_info():
    wi = _tud.get_worker_info()
    return wi


def _dataloader_autotune_on():
    from ..framework.flags import get_flags
    try:
        return bool(get_flags("FLAGS_dataloader_autotune")["FLAGS_dataloader_autotune"])
    except Exception:  # pragma: no cover
        return False


def _tune_num_workers(dataset, batch_sampler, collate, worker_init_fn):
    """Worker count with the lowest per-batch load time over the first ``FLAGS_dataloader_tuning_steps`` batches
    (at least 2 per candidate): candidates 0, 2, 4, ... up to half the visible CPUs (at most 16); a larger count
    must beat the best so far by 20 % to be taken, and the search stops at the first one that does not."""
    import os as _os
    import time as _time
    from ..framework.flags import get_flags
    try:
        steps = int(get_flags("FLAGS_dataloader_tuning_steps")["FLAGS_dataloader_tuning_steps"])
    except Exception:  # pragma: no cover
        steps = 8
    bs = getattr(batch_sampler, "batch_size", 1) or 1
    n = min(len(dataset), max(2, steps) * bs)
    sub = Subset(dataset, list(range(n)))
    sampler = BatchSampler(sub, batch_size=bs, drop_last=False)
    max_w = min(16, max(0, (len(_os.sched_getaffinity(0)) if hasattr(_os, "sched_getaffinity") else
                            (_os.cpu_count() or 2)) // 2))
    best, best_cost = 0, None
    for w in range(0, max_w + 1, 2):
        loader = _tud.DataLoader(_TorchDS(sub), batch_sampler=_BS(sampler), collate_fn=collate, num_workers=w,
                                 worker_init_fn=worker_init_fn)
        t0 = _time.perf_counter()
        cnt = sum(1 for _ in loader)
        cost = (_time.perf_counter() - t0) / max(cnt, 1)
        if best_cost is None or cost < 0.8 * best_cost:
            best, best_cost = w, cost
        elif w > best:
            break
    return best


class DataLoader:
    def __init__(self, dataset, feed_list=None, places=None, return_list=True, batch_sampler=None, batch_size=1,
                 shuffle=False, drop_last=False, collate_fn=None, num_workers=0, use_buffer_reader=True,
                 prefetch_factor=2, use_shared_memory=True, timeout=0, worker_init_fn=None, persistent_workers=False):
        self.dataset = dataset
        self.return_list = return_list
        self.collate_fn = collate_fn or default_collate_fn
        self.num_workers = num_workers
        self._iterable = isinstance(dataset, IterableDataset)
        if self._iterable:
            self.batch_sampler = None
            self.batch_size = batch_size
        else:
            if batch_sampler is None:
                batch_sampler = BatchSampler(dataset, shuffle=shuffle, batch_size=batch_size, drop_last=drop_last)
            self.batch_sampler = batch_sampler
        self.drop_last = drop_last
        self._device = _get_torch_device()
        self._pin = self._device.type == "cuda" and use_buffer_reader
        self.autotuned_num_workers = None
        if num_workers == 0 and not self._iterable and _dataloader_autotune_on():
            # FLAGS_dataloader_autotune (incubate.autotune.set_config({"dataloader": ...})): time the loader on a
            # prefix of the dataset at growing worker counts and keep the cheapest (reference io/reader.py AuToTune)
            num_workers = self.autotuned_num_workers = _tune_num_workers(
                dataset, self.batch_sampler, self._collate_np, worker_init_fn)
            self.num_workers = num_workers
        if self._iterable:
            tds = _TorchIterDS(dataset)
            self._loader = _tud.DataLoader(tds, batch_size=batch_size, drop_last=drop_last,
                                           collate_fn=self._collate_np, num_workers=num_workers,
                                           pin_memory=False, timeout=timeout, worker_init_fn=worker_init_fn,
                                           prefetch_factor=prefetch_factor if num_workers > 0 else None,
                                           persistent_workers=persistent_workers and num_workers > 0)
        else:
            tds = _TorchDS(dataset)
            self._loader = _tud.DataLoader(tds, batch_sampler=_BS(self.batch_sampler), collate_fn=self._collate_np,
                                           num_workers=num_workers, pin_memory=False, timeout=timeout,
                                           worker_init_fn=worker_init_fn,
                                           prefetch_factor=prefetch_factor if num_workers > 0 else None,
                                           persistent_workers=persistent_workers and num_workers > 0)

    def _collate_np(self, batch):
        out = self.collate_fn(batch)
        return _tensors_to_torch(out)

    def __len__(self):
        if self._iterable:
            raise TypeError("IterableDataset has no len()")
        return len(self.batch_sampler)

    def __iter__(self):
        if not self._pin:
            for b in self._loader:
                yield _wrap_out(b, self._device, False)
            return
        # use_buffer_reader: double-buffered H2D. Batch i+1 is staged through the native pinned pool
        # (device/pinned.py) and copied on a side stream while the caller computes on batch i.
        from ..device import pinned as _pinned
        dev = self._device
        side = torch.cuda.Stream(dev)

        def stage(b):
            # The staged batch is allocated on the side stream. A batch the caller has dropped went back to the
            # allocator while compute kernels queued on the current stream may still read it; record_stream
            # covers that for PyTorch's caching allocator, but a pluggable allocator (the native auto-growth
            # allocator, csrc/runtime/allocator.h) never sees record_stream and returns the block to the side
            # stream's pool at once. Ordering the side stream behind the compute stream's queued work before
            # allocating makes reuse safe under any allocator; batch i+1's copy still overlaps batch i's compute
            # (only work queued before this call, i.e. up to batch i-1, is waited for).
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                out = _stage_batch(b, dev, side, _pinned)
                ev = torch.cuda.Event()
                ev.record(side)
            return out, ev

        def release(staged):
            out, ev = staged
            cur = torch.cuda.current_stream(dev)
            cur.wait_event(ev)
            _record_stream(out, cur)
            return _wrap_out(out, None, False)

        it = iter(self._loader)
        try:
            nxt = stage(next(it))
        except StopIteration:
            return
        for b in it:
            cur = nxt
            nxt = stage(b)
            yield release(cur)
        yield release(nxt)

    def __call__(self):
        return self.__iter__()

    @staticmethod
    def from_generator(feed_list=None, capacity=None, use_double_buffer=True, iterable=True, return_list=False,
                       use_multiprocess=False, drop_last=True):
        return _GeneratorLoader()


def _tensors_to_torch(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    if isinstance(x, (list, tuple)):
        return [_tensors_to_torch(v) for v in x]
    if isinstance(x, dict):
        return {k: _tensors_to_torch(v) for k, v in x.items()}
    return x


class _GeneratorLoader:
    def __init__(self):
        self._gen = None
        self._batch = False

    def set_sample_generator(self, reader, batch_size, drop_last=True, places=None):
        def gen():
            buf = []
            for s in reader():
                buf.append(s)
                if len(buf) == batch_size:
                    yield default_collate_fn(buf)
                    buf = []
            if buf and not drop_last:
                yield default_collate_fn(buf)
        self._gen = gen

    def set_sample_list_generator(self, reader, places=None):
        self._gen = lambda: (default_collate_fn(b) for b in reader())

    def set_batch_generator(self, reader, places=None):
        self._gen = lambda: (_tensors_to_torch(b) for b in reader())

    def __iter__(self):
        dev = _get_torch_device()
        for b in self._gen():
            yield _wrap_out(b, dev, False)

    def __call__(self):
        return iter(self)
