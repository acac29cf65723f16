"""Hybrid-parallel topology. Reference: python/paddle/distributed/fleet/base/topology.py
(CommunicateTopology, HybridCommunicateGroup).

Axis order (outer -> inner) = ["data", "pipe", "sharding", "sep", "model"], like the reference: the
model-parallel (TP) ranks are contiguous. On one 8xMI355X node every GPU pair has a direct xGMI
link, so contiguity is about ring formation only; TP groups of 2 ride a single xGMI hop each.
"""
from __future__ import annotations

import collections
import itertools

import numpy as np

from .. import collective as C


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3
    SEGMENT_PARALLEL = 4


class CommunicateTopology:
    def __init__(self, hybrid_group_names=("data", "pipe", "sharding", "sep", "model"), dims=(1, 1, 1, 1, 1)):
        self._parallel_names = list(hybrid_group_names)
        self._dims = list(dims)
        self.coordinate = collections.namedtuple("Coordinate", self._parallel_names)
        self._world_size = int(np.prod(self._dims))
        ranges = [range(d) for d in self._dims]
        all_coord = [self.coordinate(*x) for x in itertools.product(*ranges)]
        self._coord2rank = dict(zip(all_coord, range(len(all_coord))))
        self._rank2coord = dict(zip(self._coord2rank.values(), self._coord2rank.keys()))

    def get_hybrid_group_names(self):
        return self._parallel_names

    def get_dim(self, axis_name):
        return self._dims[self._parallel_names.index(axis_name)]

    def world_size(self):
        return self._world_size

    def get_rank(self, **kwargs):
        return self._coord2rank[self.coordinate(**kwargs)]

    def get_coord(self, rank):
        return self._rank2coord[rank]

    def get_axis_list(self, axis_name, index):
        axis = self._parallel_names.index(axis_name)
        return sorted(r for c, r in self._coord2rank.items() if c[axis] == index)

    def get_dim_size(self, axis_name):
        return self.get_dim(axis_name)

    def get_comm_list(self, axis_name):
        """All rank groups that vary only along `axis_name`."""
        axis = self._parallel_names.index(axis_name)
        others = [range(d) for i, d in enumerate(self._dims) if i != axis]
        out = []
        for o in itertools.product(*others):
            grp = []
            for k in range(self._dims[axis]):
                coord = list(o)
                coord.insert(axis, k)
                grp.append(self._coord2rank[self.coordinate(*coord)])
            out.append(grp)
        return out

    def get_fused_ranks(self, fused_axes):
        """Rank groups that vary only along the axes in ``fused_axes`` (reference create_fuse_group)."""
        idx = [self._parallel_names.index(a) for a in fused_axes]
        groups = {}
        for c, r in self._coord2rank.items():
            key = tuple(v for i, v in enumerate(c) if i not in idx)
            groups.setdefault(key, []).append(r)
        return [sorted(g) for _, g in sorted(groups.items())]

    def get_rank_from_stage(self, global_rank, **kwargs):
        coord = self.get_coord(global_rank)._asdict()
        coord.update(kwargs)
        return self._coord2rank[self.coordinate(**coord)]


class HybridCommunicateGroup:
    def __init__(self, topology):
        self._topo = topology
        self.global_rank = C.get_rank()
        self.nranks = topology.world_size()
        self._dp_degree = topology.get_dim("data")
        self._pp_degree = topology.get_dim("pipe")
        self._sharding_degree = topology.get_dim("sharding")
        self._sep_degree = topology.get_dim("sep")
        self._mp_degree = topology.get_dim("model")
        self._groups = {}
        for axis in ("data", "pipe", "sharding", "sep", "model"):
            self._groups[axis] = self._build(axis)
        self._fused = {}
        if self._sep_degree > 1:
            self._fused[("data", "sep")] = self._build_fused(("data", "sep"))
        self.stage_id = self._topo.get_coord(self.global_rank).pipe
        # host-side (gloo) twin of the pipe groups: pipeline p2p tags / meta travel there (parallel/p2p.py)
        self._pipe_host = None
        if self._pp_degree > 1 and C.is_initialized():
            from ...parallel.p2p import host_twin
            self._pipe_host = host_twin(self._topo.get_comm_list("pipe"), self.global_rank)
        # payload twin of the pipe groups: p2p messages to a lower rank travel there (parallel/p2p.py)
        self._pipe_down = None
        if self._pp_degree > 1 and C.is_initialized():
            from ...parallel.p2p import payload_twin
            self._pipe_down = payload_twin(self._topo.get_comm_list("pipe"), self.global_rank)
        # check group for global grad-norm (all ranks that hold distinct param shards)
        self._check_group = None

    def _build(self, axis):
        mine = None
        for ranks in self._topo.get_comm_list(axis):
            if len(ranks) == 1:
                g = C.Group(0 if self.global_rank in ranks else -1, -1, ranks, None) if self.global_rank in ranks \
                    else None
            else:
                g = C.new_group(ranks) if C.is_initialized() else None
            if self.global_rank in ranks:
                mine = g if g is not None else C.Group(ranks.index(self.global_rank), -1, ranks, None)
        return mine

    def _build_fused(self, axes):
        mine = None
        for ranks in self._topo.get_fused_ranks(axes):
            g = C.new_group(ranks) if (C.is_initialized() and len(ranks) > 1) else None
            if self.global_rank in ranks:
                mine = g if g is not None else C.Group(ranks.index(self.global_rank), -1, ranks, None)
        return mine

    def get_parallel_mode(self):
        # reference order: pp -> mp -> sep -> sharding -> dp
        if self._pp_degree > 1:
            return ParallelMode.PIPELINE_PARALLEL
        if self._mp_degree > 1:
            return ParallelMode.TENSOR_PARALLEL
        if self._sep_degree > 1:
            return ParallelMode.SEGMENT_PARALLEL
        if self._sharding_degree > 1:
            return ParallelMode.SHARDING_PARALLEL
        return ParallelMode.DATA_PARALLEL

    def topology(self):
        return self._topo

    def get_global_rank(self):
        return self.global_rank

    # data
    def get_data_parallel_rank(self):
        return self._topo.get_coord(self.global_rank).data

    def get_data_parallel_world_size(self):
        return self._dp_degree

    def get_data_parallel_group(self):
        return self._groups["data"]

    def get_data_parallel_group_src_rank(self):
        return self._groups["data"].ranks[0]

    # model
    def get_model_parallel_rank(self):
        return self._topo.get_coord(self.global_rank).model

    def get_model_parallel_world_size(self):
        return self._mp_degree

    def get_model_parallel_group(self):
        return self._groups["model"]

    def get_model_parallel_group_src_rank(self):
        return self._groups["model"].ranks[0]

    # pipe
    def get_stage_id(self):
        return self.stage_id

    def get_pipe_parallel_world_size(self):
        return self._pp_degree

    def get_pipe_parallel_group(self):
        return self._groups["pipe"]

    def get_pipe_parallel_host_group(self):
        """gloo twin of this rank's pipe group (headers and tags of pipeline p2p travel there)."""
        return self._pipe_host

    def get_pipe_parallel_down_group(self):
        """Second payload group of this rank's pipe group (messages to a lower rank; parallel/p2p.py)."""
        return self._pipe_down

    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self._pp_degree - 1

    # sharding
    def get_sharding_parallel_rank(self):
        return self._topo.get_coord(self.global_rank).sharding

    def get_sharding_parallel_world_size(self):
        return self._sharding_degree

    def get_sharding_parallel_group(self):
        return self._groups["sharding"]

    def get_sharding_parallel_group_src_rank(self):
        return self._groups["sharding"].ranks[0]

    # sep
    def get_sep_parallel_rank(self):
        return self._topo.get_coord(self.global_rank).sep

    def get_sep_parallel_world_size(self):
        return self._sep_degree

    def get_sep_parallel_group(self):
        return self._groups["sep"]

    def get_sep_parallel_group_src_rank(self):
        return self._groups["sep"].ranks[0]

    def get_dp_sep_parallel_group(self):
        """data x sep fused group (gradients of sep-parallel training are reduced over it)."""
        if self._sep_degree <= 1:
            return self._groups["data"]
        return self._fused[("data", "sep")]

    def get_check_parallel_group(self, sharding=False):
        return None

    def get_rank_from_stage(self, stage_id, **kwargs):
        return self._topo.get_rank_from_stage(self.global_rank, pipe=stage_id, **kwargs)


_HCG = None


def _set_hcg(h):
    global _HCG
    _HCG = h


def _get_hcg():
    return _HCG
