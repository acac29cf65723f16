"""Placements. Reference: python/paddle/distributed/auto_parallel/placement_type.py (Shard, Replicate,
Partial, ReduceType). Each maps 1:1 onto the device-tensor placement used by the SPMD runtime."""
from __future__ import annotations

from torch.distributed import tensor as _dt


class ReduceType:
    kRedSum = 0
    kRedMax = 1
    kRedMin = 2
    kRedProd = 3
    kRedAvg = 4
    kRedAny = 5
    kRedAll = 6


_RED = {ReduceType.kRedSum: "sum", ReduceType.kRedAvg: "avg", ReduceType.kRedMax: "max", ReduceType.kRedMin: "min",
        ReduceType.kRedProd: "product"}


class Placement:
    def is_shard(self, dim=None):
        return False

    def is_replicated(self):
        return False

    def is_partial(self):
        return False


class Shard(Placement):
    def __init__(self, dim, shard_order=None, split_factor=1):
        self.dim = int(dim)

    def get_dim(self):
        return self.dim

    def is_shard(self, dim=None):
        return dim is None or dim == self.dim

    def _to_torch(self):
        return _dt.Shard(self.dim)

    def __eq__(self, o):
        return isinstance(o, Shard) and o.dim == self.dim

    def __hash__(self):
        return hash(("shard", self.dim))

    def __repr__(self):
        return f"Shard(dim={self.dim})"


class Replicate(Placement):
    def is_replicated(self):
        return True

    def _to_torch(self):
        return _dt.Replicate()

    def __eq__(self, o):
        return isinstance(o, Replicate)

    def __hash__(self):
        return hash("replicate")

    def __repr__(self):
        return "Replicate()"


class Partial(Placement):
    def __init__(self, reduce_type=ReduceType.kRedSum):
        self.reduce_type = reduce_type

    def is_partial(self):
        return True

    def _to_torch(self):
        return _dt.Partial(_RED.get(self.reduce_type, "sum"))

    def __eq__(self, o):
        return isinstance(o, Partial) and o.reduce_type == self.reduce_type

    def __hash__(self):
        return hash(("partial", self.reduce_type))

    def __repr__(self):
        return f"Partial(reduce_type={self.reduce_type})"


def to_torch_placements(placements):
    return [p._to_torch() for p in placements]


def from_torch_placements(pls):
    out = []
    for p in pls:
        if isinstance(p, _dt.Shard):
            out.append(Shard(p.dim))
        elif isinstance(p, _dt.Partial):
            inv = {v: k for k, v in _RED.items()}
            out.append(Partial(inv.get(getattr(p, "reduce_op", "sum"), ReduceType.kRedSum)))
        else:
            out.append(Replicate())
    return out
