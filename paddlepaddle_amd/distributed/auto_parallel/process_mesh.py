"""ProcessMesh. Reference: python/paddle/distributed/auto_parallel/process_mesh.py.

A ProcessMesh is an N-d array of global ranks with named dims. Its runtime form is a device mesh whose
per-dim process groups are RCCL communicators (one per mesh row/column) — on an 8xMI355X node every
pair of GPUs has its own xGMI link, so any 2-D factorisation (e.g. 2x4 dp x mp) keeps each collective
on direct links. The device mesh is built lazily, the first time a distributed tensor needs it.
"""
from __future__ import annotations

import numpy as np
import torch

_current = []


class ProcessMesh:
    def __init__(self, mesh=None, dim_names=None, shape=None, process_ids=None):
        if mesh is None:
            mesh = np.asarray(process_ids).reshape(shape)
        self._mesh = np.asarray(mesh, dtype=np.int64)
        if self._mesh.ndim == 0:
            self._mesh = self._mesh.reshape(1)
        self._dim_names = list(dim_names) if dim_names is not None else [f"d{i}" for i in range(self._mesh.ndim)]
        assert len(self._dim_names) == self._mesh.ndim
        self._device_mesh = None

    @property
    def mesh(self):
        return self._mesh

    @property
    def shape(self):
        return list(self._mesh.shape)

    @property
    def ndim(self):
        return self._mesh.ndim

    @property
    def dim_names(self):
        return list(self._dim_names)

    @property
    def process_ids(self):
        return self._mesh.flatten().tolist()

    def get_dim_size(self, dim):
        if isinstance(dim, str):
            dim = self._dim_names.index(dim)
        return self._mesh.shape[dim]

    def get_mesh_with_dim(self, dim_name, index=None):
        ax = self._dim_names.index(dim_name)
        m = np.moveaxis(self._mesh, ax, 0)
        names = [dim_name] + [n for n in self._dim_names if n != dim_name]
        if index is not None:
            return ProcessMesh(m[index], names[1:])
        return ProcessMesh(m, names)

    def get_submesh_with_dim(self, dim_name):
        from .. import collective as C
        r = C.get_rank()
        ax = self._dim_names.index(dim_name)
        coord = np.argwhere(self._mesh == r)
        if coord.size == 0:
            return None
        idx = list(coord[0])
        sl = [i for i in idx]
        sl[ax] = slice(None)
        return ProcessMesh(self._mesh[tuple(sl)], [dim_name])

    def __getitem__(self, idx):
        sub = self._mesh[idx]
        if isinstance(idx, (int, np.integer)):
            names = self._dim_names[1:]
        elif isinstance(idx, tuple):
            names = [n for i, n in enumerate(self._dim_names) if i >= len(idx) or isinstance(idx[i], slice)]
        else:
            names = self._dim_names
        return ProcessMesh(sub, names if sub.ndim == len(names) else None)

    def contains(self, rank):
        return rank in self.process_ids

    def __contains__(self, rank):
        return self.contains(rank)

    def __eq__(self, o):
        return isinstance(o, ProcessMesh) and np.array_equal(o._mesh, self._mesh) and o._dim_names == self._dim_names

    def __hash__(self):
        return hash((self._mesh.tobytes(), tuple(self._mesh.shape), tuple(self._dim_names)))

    def __repr__(self):
        return f"ProcessMesh(shape={self.shape}, process_ids={self.process_ids}, dim_names={self._dim_names})"

    def __enter__(self):
        _current.append(self)
        return self

    def __exit__(self, *a):
        _current.pop()

    # ------------------------------------------------------------------ runtime
    def _dev_type(self):
        from ...framework.place import _get_torch_device
        return "cuda" if _get_torch_device().type == "cuda" else "cpu"

    def device_mesh(self):
        if self._device_mesh is None:
            from torch.distributed.device_mesh import DeviceMesh
            from .. import collective as C
            if not C.is_initialized():
                C.init_parallel_env()
            self._device_mesh = DeviceMesh(self._dev_type(), torch.as_tensor(self._mesh),
                                           mesh_dim_names=tuple(self._dim_names))
        return self._device_mesh


_global_mesh = [None]


def get_mesh():
    return _global_mesh[0]


def set_mesh(mesh):
    _global_mesh[0] = mesh


def get_current_process_mesh():
    return _current[-1] if _current else None
