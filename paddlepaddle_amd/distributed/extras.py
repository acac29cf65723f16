"""Remaining paddle.distributed names: gloo helpers, ParallelMode, DistAttr, split (model-parallel layer
builder), distributed.io (persistables save/load), and the parameter-server dataset / sparse-table entry
classes.

Reference: python/paddle/distributed/__init__.py, parallel_with_gloo.py (gloo_init_parallel_env /
gloo_barrier / gloo_release), fleet/layers/mpu/mp_ops.py:split, io.py, fleet/dataset/dataset.py
(InMemoryDataset / QueueDataset), entry_attr.py. The parameter-server stack (D13) is out of scope on a
GPU node: the dataset classes keep the reference's configuration API and feed local files through
paddle.io, the sparse-table entries are plain config records.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

__all__ = ["gloo_init_parallel_env", "gloo_barrier", "gloo_release", "ParallelMode", "DistAttr", "split", "io",
           "InMemoryDataset", "QueueDataset", "ProbabilityEntry", "CountFilterEntry", "ShowClickEntry"]

_GLOO = {}


def gloo_init_parallel_env(rank_id, rank_num, server_endpoint):
    """A CPU (gloo) process group used for host-side barriers, independent of the RCCL group."""
    host, port = server_endpoint.split(":")
    store = dist.TCPStore(host, int(port), rank_num, rank_id == 0)
    _GLOO["store"] = store
    if not dist.is_initialized():
        dist.init_process_group("gloo", store=store, rank=rank_id, world_size=rank_num)
        _GLOO["pg"] = None
    else:
        _GLOO["pg"] = dist.new_group(list(range(rank_num)), backend="gloo")
    _GLOO["rank"], _GLOO["n"] = rank_id, rank_num


def gloo_barrier():
    if "rank" not in _GLOO:
        raise RuntimeError("call gloo_init_parallel_env first")
    dist.barrier(group=_GLOO.get("pg"))


def gloo_release():
    if _GLOO.get("pg") is None and dist.is_initialized() and "rank" in _GLOO:
        dist.destroy_process_group()
    _GLOO.clear()


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3
    SEGMENT_PARALLEL = 4


class DistAttr:
    """Static auto-parallel tensor annotation: a ProcessMesh + per-dim mesh-axis names (None = replicated)."""

    def __init__(self, mesh, sharding_specs):
        self.process_mesh = mesh
        self.sharding_specs = list(sharding_specs)
        names = getattr(mesh, "dim_names", None) or []
        self.dims_mapping = [names.index(s) if s is not None and s in names else -1 for s in self.sharding_specs]

    def __repr__(self):
        return f"DistAttr(mesh={self.process_mesh}, sharding_specs={self.sharding_specs})"


def split(x, size, operation, axis=0, num_partitions=1, gather_out=True, weight_attr=None, bias_attr=None,
          name=None):
    """Model-parallel linear / embedding over the model-parallel group (reference mp_ops.split):
    operation 'linear' splits the weight along ``axis`` (0 = row parallel, 1 = column parallel),
    'embedding' splits the vocabulary."""
    from ..parallel import tensor_parallel as M
    if operation == "embedding":
        layer = M.VocabParallelEmbedding(size[0], size[1], weight_attr=weight_attr)
        return layer(x)
    if operation == "linear":
        if axis == 1:
            layer = M.ColumnParallelLinear(size[0], size[1], weight_attr=weight_attr, has_bias=bias_attr is not False,
                                           gather_output=gather_out)
        else:
            layer = M.RowParallelLinear(size[0], size[1], weight_attr=weight_attr, has_bias=bias_attr is not False,
                                        input_is_parallel=False)
        return layer(x)
    raise ValueError(f"unsupported operation {operation!r} (linear | embedding)")


class _IO:
    """paddle.distributed.io: persistables of a (static) program on rank 0's filesystem."""

    @staticmethod
    def save_persistables(executor, dirname, main_program=None, filename=None):
        from ..static.io import save_persistables
        return save_persistables(executor, dirname, main_program, filename)

    @staticmethod
    def load_persistables(executor, dirname, main_program=None, filename=None):
        from ..static.io import load_persistables
        return load_persistables(executor, dirname, main_program, filename)

    @staticmethod
    def is_persistable(var):
        return bool(getattr(var, "persistable", False))

    @staticmethod
    def load_inference_model_distributed(dirname=None, executor=None, model_filename=None, params_filename=None,
                                         pserver_endpoints=None, path_prefix=None, **kw):
        """A program saved by (fluid) save_inference_model under ``dirname``; ``pserver_endpoints`` name the
        servers of distributed lookup tables, which this framework's programs read through their own PS
        runtime (distributed/ps), so they need no rewrite here."""
        from ..base.io import load_inference_model
        if path_prefix is not None:
            return load_inference_model(path_prefix, executor, **kw)
        return load_inference_model(executor=executor, dirname=dirname, model_filename=model_filename, **kw)


io = _IO()


class _DatasetBase:
    """Configuration surface of the PS datasets; records are read from local text files with a user
    `parse_fn(line) -> sample` (set_parse_fn) and served through paddle.io."""

    def __init__(self):
        self.filelist, self.batch_size, self.thread_num, self.use_var = [], 1, 1, []
        self.pipe_command, self._parse = "cat", None
        self._records = None

    def init(self, batch_size=1, thread_num=1, use_var=None, pipe_command="cat", input_type=0, fs_name="",
             fs_ugi="", download_cmd="cat", **kwargs):
        self.batch_size, self.thread_num, self.use_var, self.pipe_command = batch_size, thread_num, use_var or [], \
            pipe_command

    def set_filelist(self, filelist):
        self.filelist = list(filelist)

    def set_parse_fn(self, fn):
        self._parse = fn

    def _iter_lines(self):
        for f in self.filelist:
            with open(f) as fh:
                for line in fh:
                    yield self._parse(line) if self._parse else line.rstrip("\n")

    def __iter__(self):
        batch = []
        for r in (self._records if self._records is not None else self._iter_lines()):
            batch.append(r)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if batch:
            yield batch


class QueueDataset(_DatasetBase):
    pass


class InMemoryDataset(_DatasetBase):
    def load_into_memory(self, is_shuffle=False):
        self._records = list(self._iter_lines())

    def local_shuffle(self):
        import random
        random.shuffle(self._records)

    def global_shuffle(self, fleet=None, thread_num=12):
        self.local_shuffle()

    def release_memory(self):
        self._records = None

    def get_memory_data_size(self, fleet=None):
        return len(self._records or [])

    def get_shuffle_data_size(self, fleet=None):
        return self.get_memory_data_size()


class _Entry:
    def __init__(self, *args):
        self._args = args

    def _to_attr(self):
        return ":".join([self._name] + [str(a) for a in self._args])


class ProbabilityEntry(_Entry):
    _name = "probability_entry"

    def __init__(self, probability):
        if not 0 < probability <= 1:
            raise ValueError("probability must be in (0, 1]")
        super().__init__(probability)


class CountFilterEntry(_Entry):
    _name = "count_filter_entry"

    def __init__(self, count_filter):
        if count_filter < 0:
            raise ValueError("count_filter must be >= 0")
        super().__init__(count_filter)


class ShowClickEntry(_Entry):
    _name = "show_click_entry"

    def __init__(self, show_name, click_name):
        super().__init__(show_name, click_name)
