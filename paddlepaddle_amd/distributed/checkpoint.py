"""Distributed checkpoint with reshard-on-load.

Reference: python/paddle/distributed/checkpoint/{save_state_dict.py,load_state_dict.py,metadata.py}.

Layout of a checkpoint directory:
  ``{rank}_0.distcp``  safetensors file per rank holding that rank's *unique* local chunks
  ``0.metadata``       JSON: for every key its global shape/dtype and the list of chunks
                       (file, tensor name, global offset, local shape) — written by the coordinator
Load computes, for every key of the *target* state dict (any world size / placements), the global
box its local shard covers, and copies in the intersecting pieces of the saved chunks (read lazily
with safetensors; nothing is unpickled). Replicated values are written once (by the lowest rank
holding them), so a checkpoint's size is the model size, not world x model size.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from ..framework.tensor import Tensor
from . import collective as C


def _flatten(sd, prefix=""):
    out = {}
    for k, v in sd.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(_flatten(v, key + "."))
        else:
            out[key] = v
    return out


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
    return t, tuple(t.shape), tuple(0 for _ in t.shape), C.get_rank() == 0 if C.is_initialized() else True


def save_state_dict(state_dict, path, process_group=None, coordinator_rank=0, unique_id=None, async_save=False):
    os.makedirs(path, exist_ok=True)
    from safetensors.torch import save_file
    rank = C.get_rank() if C.is_initialized() else 0
    flat = _flatten(state_dict)
    tensors, chunks = {}, {}
    fname = f"{rank}_0.distcp"
    for k, v in flat.items():
        if isinstance(v, (int, float, str, bool)) or v is None:
            chunks[k] = {"scalar": v}
            continue
        t = v._t if isinstance(v, Tensor) else (v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v)))
        local, gshape, off, primary = _local_box(t)
        meta = {"global_shape": list(gshape), "dtype": str(local.dtype).replace("torch.", ""), "chunks": []}
        if primary and local.numel() > 0:
            name = f"{k}@{'_'.join(map(str, off))}"
            tensors[name] = local.detach().contiguous().cpu()
            meta["chunks"].append({"file": fname, "name": name, "offset": list(off), "shape": list(local.shape)})
        chunks[k] = meta
    save_file(tensors, os.path.join(path, fname))
    # gather chunk lists on the coordinator and merge
    if C.is_initialized() and C.get_world_size() > 1:
        allm = []
        C.all_gather_object(allm, chunks)
    else:
        allm = [chunks]
    if rank == coordinator_rank:
        merged = {}
        for m in allm:
            for k, meta in m.items():
                if "scalar" in meta:
                    merged.setdefault(k, meta)
                    continue
                cur = merged.setdefault(k, {"global_shape": meta["global_shape"], "dtype": meta["dtype"], "chunks": []})
                cur["chunks"].extend(meta["chunks"])
        with open(os.path.join(path, "0.metadata"), "w") as f:
            json.dump({"version": 1, "state": merged}, f)
    if C.is_initialized() and C.get_world_size() > 1:
        C.barrier()


def _intersect(a_off, a_shape, b_off, b_shape):
    lo = [max(x, y) for x, y in zip(a_off, b_off)]
    hi = [min(x + s, y + t) for x, s, y, t in zip(a_off, a_shape, b_off, b_shape)]
    if any(h <= l for l, h in zip(lo, hi)):
        return None
    return lo, hi


def load_state_dict(state_dict, path, process_group=None, coordinator_rank=0, unique_id=None, offload=False):
    """Fill ``state_dict``'s tensors in place from the checkpoint, whatever their sharding now is."""
    from safetensors import safe_open
    with open(os.path.join(path, "0.metadata")) as f:
        meta = json.load(f)["state"]
    flat = _flatten(state_dict)
    handles = {}

    def h(fn):
        if fn not in handles:
            handles[fn] = safe_open(os.path.join(path, fn), framework="pt")
        return handles[fn]
    missing = []
    for k, v in flat.items():
        if k not in meta:
            missing.append(k)
            continue
        m = meta[k]
        if "scalar" in m:
            continue
        t = v._t if isinstance(v, Tensor) else v
        if not isinstance(t, torch.Tensor):
            continue
        local, gshape, off, _ = _local_box(t)
        if list(gshape) != list(m["global_shape"]):
            raise ValueError(f"{k}: checkpoint global shape {m['global_shape']} != target {list(gshape)}")
        with torch.no_grad():
            for c in m["chunks"]:
                box = _intersect(off, local.shape, c["offset"], c["shape"])
                if box is None:
                    continue
                lo, hi = box
                src = h(c["file"]).get_slice(c["name"])
                sl_src = tuple(slice(l - o, hh - o) for l, hh, o in zip(lo, hi, c["offset"]))
                piece = src[sl_src] if len(sl_src) else h(c["file"]).get_tensor(c["name"])
                sl_dst = tuple(slice(l - o, hh - o) for l, hh, o in zip(lo, hi, off))
                dst = local[sl_dst] if len(sl_dst) else local
                dst.copy_(piece.to(dst.dtype))
    if missing:
        import warnings
        warnings.warn(f"load_state_dict: keys not in checkpoint: {missing[:8]}{'...' if len(missing) > 8 else ''}")
    return state_dict


def get_checkpoint_files(path, use_dist=False):
    return sorted(f for f in os.listdir(path) if f.endswith(".distcp") or f.endswith(".metadata"))
