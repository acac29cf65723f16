"""Distributed checkpoint in the reference on-disk layout, with reshard-on-load.

Reference: python/paddle/distributed/checkpoint/{save_state_dict.py:278,311, load_state_dict.py, metadata.py,
utils.py}.

A checkpoint directory holds
  ``{rank}_{uid}.distcp``  ``paddle.save`` of that rank's local chunks {flat key: tensor} (replicated tensors are
                           kept by one rank only), readable by paddle.load / framework.io.load;
  ``{uid}.metadata``       ``paddle.save`` of a ``Metadata``: per flat key the chunks (global offset, local shape,
                           dtype name), per chunk the file holding it, and the flat-key -> nested-key mapping.
Files written here load in PaddlePaddle and vice versa. Loading computes, for every key of the *target* state
dict (any world size / placement), the global box its local shard covers and copies the intersecting parts of
the saved chunks in; .distcp files are read once each and only by ranks that need a chunk from them.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

from ...framework.tensor import Tensor
from .. import collective as C
from .metadata import LocalTensorIndex, LocalTensorMetadata, Metadata, PICKLE_MODULE

__all__ = ["save_state_dict", "load_state_dict", "get_checkpoint_files", "Metadata", "LocalTensorMetadata",
           "LocalTensorIndex"]


# ------------------------------------------------------------------------------------------------ helpers
def flatten_state_dict(state_dict):
    """{"model": {"w0": t}} -> ({"model.w0": t}, {"model.w0": ("model", "w0")}) (reference utils.py)."""
    flat, mapping = {}, {}

    def rec(key, value):
        if isinstance(value, dict):
            for k, v in value.items():
                if not isinstance(k, str):
                    raise ValueError(f"The key should be str, but is {k}")
                rec((*key, k), v)
        else:
            s = ".".join(key)
            flat[s] = value
            mapping[s] = key
    rec((), state_dict)
    return flat, mapping


def _torch(v):
    if isinstance(v, Tensor):
        return v._t
    if isinstance(v, torch.Tensor):
        return v
    return torch.as_tensor(np.asarray(v))


def _local_box(t):
    """(local tensor, global shape, global offset, is_primary_copy) for plain or distributed tensors."""
    from torch.distributed.tensor import DTensor
    if isinstance(t, DTensor):
        from torch.distributed.tensor._utils import compute_local_shape_and_global_offset
        shape, offset = compute_local_shape_and_global_offset(t.shape, t.device_mesh, t.placements)
        local = t.to_local()
        coord = t.device_mesh.get_coordinate()
        primary = True
        for i, p in enumerate(t.placements):
            if not p.is_shard() and coord is not None and coord[i] != 0:
                primary = False  # replicated / partial along this mesh dim: only index 0 writes
        return local, tuple(t.shape), tuple(offset), primary
    sharded = getattr(t, "_pa_global", None)  # (global_shape, offset) annotated by sharding engines
    if sharded is not None:
        return t, tuple(sharded[0]), tuple(sharded[1]), True
    return t, tuple(t.shape), tuple(0 for _ in t.shape), True


def _dtype_name(t):
    return str(t.dtype).replace("torch.", "")


class _PaddleModuleAlias:
    """While pickling Metadata, make ``paddle.distributed.checkpoint.metadata`` importable as this package's
    metadata module (unless a real ``paddle`` is loaded), so the file names the reference classes."""

    def __enter__(self):
        self.added = []
        from . import metadata as mod
        if "paddle" in sys.modules and not getattr(sys.modules["paddle"], "_pa_alias", False):
            real = sys.modules.get(PICKLE_MODULE)
            if real is not None and all(getattr(real, n, None) is getattr(mod, n) for n in mod.CLASSES):
                return self
        parts = PICKLE_MODULE.split(".")
        for i in range(1, len(parts) + 1):
            name = ".".join(parts[:i])
            if name not in sys.modules:
                m = mod if i == len(parts) else types.ModuleType(name)
                m._pa_alias = True
                sys.modules[name] = m
                self.added.append(name)
        return self

    def __exit__(self, *exc):
        for name in self.added:
            sys.modules.pop(name, None)
        return False


def _rank(group):
    if not C.is_initialized():
        return 0
    return C.get_rank()


# ------------------------------------------------------------------------------------------------ save
def save_state_dict(state_dict, path, process_group=None, coordinator_rank=0, unique_id=None, async_save=False):
    """Write this rank's chunks to ``{rank}_{uid}.distcp`` and (coordinator) the merged ``{uid}.metadata``."""
    from ...framework.io import save as _save
    os.makedirs(path, exist_ok=True)
    rank = _rank(process_group)
    multi = C.is_initialized() and C.get_world_size() > 1
    if unique_id is None:
        uid = 0
        while os.path.exists(os.path.join(path, f"{rank}_{uid}.distcp")):
            uid += 1
        if multi:  # every rank must use the same id: the largest any rank needs
            ids = []
            C.all_gather_object(ids, uid)
            uid = max(ids)
    else:
        uid = int(unique_id)
    file_name = f"{rank}_{uid}.distcp"
    flat, mapping = flatten_state_dict(state_dict)
    local_sd, local_meta, local_storage = {}, {}, {}
    for key, val in flat.items():
        t = _torch(val)
        local, gshape, off, primary = _local_box(t)
        if local.numel() == 0 and len(gshape) > 0:
            continue
        local_meta[key] = LocalTensorMetadata(tuple(off), tuple(local.shape), _dtype_name(local))
        local_storage[LocalTensorIndex(key, tuple(off))] = file_name if primary else None
        if primary:
            local_sd[key] = Tensor(local.detach())
    if multi:  # exchanged as plain tuples; the records are rebuilt below
        gathered = []
        C.all_gather_object(gathered, ({k: (m.global_offset, m.local_shape, m.dtype) for k, m in local_meta.items()},
                                       {(i.tensor_key, i.global_offset): fn for i, fn in local_storage.items()},
                                       mapping))
        all_meta = [{k: LocalTensorMetadata(*v) for k, v in g[0].items()} for g in gathered]
        all_storage = [{LocalTensorIndex(*i): fn for i, fn in g[1].items()} for g in gathered]
        all_map = [g[2] for g in gathered]
    else:
        all_meta, all_storage, all_map = [local_meta], [local_storage], [mapping]
    md = Metadata(state_dict_metadata={}, storage_metadata={}, flat_mapping={})
    for m in all_meta:
        for k, lm in m.items():
            lst = md.state_dict_metadata.setdefault(k, [])
            if all(x.global_offset != lm.global_offset for x in lst):
                lst.append(lm)
    for st in all_storage:  # the first (lowest) rank holding a chunk stores it
        for idx, fn in st.items():
            if fn is not None and idx not in md.storage_metadata:
                md.storage_metadata[idx] = fn
    for m in all_map:
        md.flat_mapping.update(m)
    # dedup: a replicated chunk that another rank stores is dropped here
    for idx, fn in md.storage_metadata.items():
        if idx.tensor_key in local_sd and idx.global_offset == local_meta[idx.tensor_key].global_offset \
                and fn != file_name:
            local_sd.pop(idx.tensor_key)
    if rank == coordinator_rank:
        with _PaddleModuleAlias():
            _save(md, os.path.join(path, f"{uid}.metadata"))
    _save(local_sd, os.path.join(path, file_name))
    if multi:
        C.barrier()


# ------------------------------------------------------------------------------------------------ load
def _intersect(a_off, a_shape, b_off, b_shape):
    lo = [max(x, y) for x, y in zip(a_off, b_off)]
    hi = [min(x + s, y + t) for x, s, y, t in zip(a_off, a_shape, b_off, b_shape)]
    if any(h <= l for l, h in zip(lo, hi)):
        return None
    return lo, hi


def _read_metadata(path, unique_id):
    from ...framework.io import load as _load
    names = sorted(f for f in os.listdir(path) if f.endswith(".metadata"))
    if not names:
        raise FileNotFoundError(f"No metadata file found in the checkpoint directory:{path}.")
    if unique_id is not None:
        names = [f"{unique_id}.metadata"]
    else:  # the newest checkpoint in the directory
        names = [max(names, key=lambda n: int(n.split(".")[0]) if n.split(".")[0].isdigit() else -1)]
    return _load(os.path.join(path, names[0]), return_numpy=True), names[0].split(".")[0]


def load_state_dict(state_dict, path, process_group=None, coordinator_rank=0, unique_id=None, offload=False):
    """Fill ``state_dict``'s tensors in place from the checkpoint, whatever their sharding now is."""
    from ...framework.io import load as _load
    md, _ = _read_metadata(path, unique_id)
    flat, _ = flatten_state_dict(state_dict)
    cache = {}

    def chunk(file_name, key):
        if file_name not in cache:
            cache[file_name] = _load(os.path.join(path, file_name), return_numpy=True)
        return cache[file_name][key]
    missing = []
    for key, val in flat.items():
        metas = md.state_dict_metadata.get(key)
        if metas is None:
            missing.append(key)
            continue
        t = _torch(val)
        local, gshape, off, _ = _local_box(t)
        with torch.no_grad():
            for lm in metas:
                box = _intersect(off, local.shape, lm.global_offset, lm.local_shape)
                if box is None and len(local.shape) > 0:
                    continue
                fn = md.storage_metadata.get(LocalTensorIndex(key, tuple(lm.global_offset)))
                if fn is None:
                    continue
                arr = chunk(fn, key)
                src = torch.from_numpy(np.ascontiguousarray(arr))
                if lm.dtype == "bfloat16" and src.dtype == torch.int16 or arr.dtype == np.uint16:
                    src = torch.from_numpy(np.ascontiguousarray(arr).view(np.int16)).view(torch.bfloat16)
                if len(local.shape) == 0:
                    local.copy_(src.reshape(()).to(local.dtype))
                    continue
                lo, hi = box
                piece = src[tuple(slice(l - o, h - o) for l, h, o in zip(lo, hi, lm.global_offset))]
                dst = local[tuple(slice(l - o, h - o) for l, h, o in zip(lo, hi, off))]
                dst.copy_(piece.to(device=dst.device, dtype=dst.dtype))
    if missing:
        import warnings
        warnings.warn(f"load_state_dict: keys not in checkpoint: {missing[:8]}{'...' if len(missing) > 8 else ''}")
    return state_dict


def get_checkpoint_files(path, use_dist=False):
    return sorted(f for f in os.listdir(path) if f.endswith(".distcp") or f.endswith(".metadata"))
