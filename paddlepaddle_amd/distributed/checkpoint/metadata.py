"""Checkpoint metadata records. Reference: python/paddle/distributed/checkpoint/metadata.py (same classes and
fields, so a ``{uid}.metadata`` file pickles / unpickles identically on both sides).

The classes report ``paddle.distributed.checkpoint.metadata`` as their module: a metadata file written here
names the reference classes (PaddlePaddle reads it natively) and one written by PaddlePaddle resolves to these
(the restricted loader of framework/io.py maps exactly these three names, nothing else)."""
from __future__ import annotations

from dataclasses import dataclass

PICKLE_MODULE = "paddle.distributed.checkpoint.metadata"


@dataclass
class LocalTensorMetadata:
    """The location of a local tensor in the global tensor."""
    global_offset: tuple
    local_shape: tuple
    dtype: str


@dataclass(frozen=True)
class LocalTensorIndex:
    """The identifier of a local tensor."""
    tensor_key: str
    global_offset: tuple


@dataclass
class Metadata:
    state_dict_metadata: dict = None
    storage_metadata: dict = None
    flat_mapping: dict = None


for _c in (LocalTensorMetadata, LocalTensorIndex, Metadata):
    _c.__module__ = PICKLE_MODULE

CLASSES = {c.__name__: c for c in (LocalTensorMetadata, LocalTensorIndex, Metadata)}
