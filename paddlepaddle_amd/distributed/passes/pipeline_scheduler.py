"""Pipeline scheduler passes (reference: python/paddle/distributed/passes/pipeline_scheduler_pass/ —
pipeline_fthenb.py, pipeline_1f1b.py, pipeline_eager_1f1b.py, pipeline_zero_bubble.py:61 ZBH1, pipeline_vpp.py).

The reference passes split a stage's program into forward / backward / optimizer sub-programs and build the
job list its standalone executor walks. Here a stage program is partitioned by the static auto-parallel engine
(distributed/auto_parallel/static_engine.py), which runs forward / backward / weight-gradient jobs of each
micro-batch itself; the pass supplies the job list: it reads ``num_micro_batches``, ``pp_stage``, ``pp_degree``
(and ``vpp_degree`` for VPP), builds the stage's jobs from parallel/pp_schedules.py (the same lists the dygraph
fleet pipelines run) and stores them as ``context.get_attr("pipeline_scheduler.job_list")`` and on the program
(``program._pa_jobs``). The engine obtains its jobs through these passes (``strategy.pipeline.schedule_mode``).
"""
from __future__ import annotations

from .pass_base import PassBase, PassType, register_pass
from ...parallel import pp_schedules as PS

__all__ = ["Job", "PipelineFThenBPass", "Pipeline1F1BPass", "PipelineEager1F1BPass", "PipelineZBH1Pass",
           "PipelineVPPPass", "PipelineZBVPPPass"]

FORWARD, BACKWARD, BACKWARD_W, OPT = "forward", "backward", "backward_w", "optimizer"
_KIND = {"F": FORWARD, "B": BACKWARD, "W": BACKWARD_W}


class Job:
    """One scheduled unit (reference core.Job): type forward / backward / backward_w / optimizer, the micro-batch
    it runs and, for VPP, the model chunk."""

    __slots__ = ("_type", "_mb", "_chunk")

    def __init__(self, type_, micro_batch_id=0, chunk_id=0):
        self._type, self._mb, self._chunk = type_, int(micro_batch_id), int(chunk_id)

    def type(self):
        return self._type

    def micro_batch_id(self):
        return self._mb

    def set_micro_batch_id(self, mb):
        self._mb = int(mb)

    def chunk_id(self):
        return self._chunk

    def as_tuple(self):
        return {FORWARD: "F", BACKWARD: "B", BACKWARD_W: "W"}.get(self._type, "O"), self._mb

    def __repr__(self):
        return f"Job({self._type}, mb={self._mb}" + (f", chunk={self._chunk})" if self._chunk else ")")

    def __eq__(self, other):
        return isinstance(other, Job) and (self._type, self._mb, self._chunk) == (other._type, other._mb,
                                                                                   other._chunk)


class _PipelinePassBase(PassBase):
    _mode = None

    def _type(self):
        return PassType.PARALLEL_OPT

    def _check_self(self):
        n, s, d = (self.get_attr(k) for k in ("num_micro_batches", "pp_stage", "pp_degree"))
        return n is not None and s is not None and d is not None and 0 <= int(s) < int(d) and int(n) >= 1

    def _pairs(self, n, s, d):
        return PS.schedule(self._mode, d, s, n)

    def _create_job_list(self):
        n, s, d = (int(self.get_attr(k)) for k in ("num_micro_batches", "pp_stage", "pp_degree"))
        jobs = [Job(_KIND[k], mb) for k, mb in self._pairs(n, s, d)]
        jobs.append(Job(OPT))
        return jobs

    def _apply_single_impl(self, prog, startup, context):
        jobs = self._create_job_list()
        prog._pa_jobs = jobs
        context.set_attr("pipeline_scheduler.job_list", jobs)
        context.set_attr("pipeline_scheduler.mode", self._mode)


@register_pass("pipeline_scheduler_FThenB")
class PipelineFThenBPass(_PipelinePassBase):
    _mode = "FTHENB"


@register_pass("pipeline_scheduler_1F1B")
class Pipeline1F1BPass(_PipelinePassBase):
    _mode = "1F1B"


@register_pass("pipeline_scheduler_Eager1F1B")
class PipelineEager1F1BPass(_PipelinePassBase):
    _mode = "EAGER1F1B"


@register_pass("pipeline_scheduler_ZBH1")
class PipelineZBH1Pass(_PipelinePassBase):
    _mode = "ZBH1"


@register_pass("pipeline_scheduler_VPP")
class PipelineVPPPass(_PipelinePassBase):
    """Interleaved 1F1B over ``vpp_degree`` chunks per stage; jobs carry (micro-batch, chunk)."""
    _mode = "VPP"

    def _check_self(self):
        return super()._check_self() and int(self.get_attr("vpp_degree", 1)) >= 1 and \
            int(self.get_attr("num_micro_batches")) % int(self.get_attr("pp_degree")) == 0

    def _create_job_list(self):
        n, s, d = (int(self.get_attr(k)) for k in ("num_micro_batches", "pp_stage", "pp_degree"))
        v = int(self.get_attr("vpp_degree", 1))
        jobs = [Job(_KIND[k], PS.vpp_mb(i, d, v), PS.vpp_chunk(i, d, v, k == "F")) for k, i in PS.vpp(d, s, n, v)]
        jobs.append(Job(OPT))
        return jobs


@register_pass("pipeline_scheduler_ZBVPP")
class PipelineZBVPPPass(PipelineVPPPass):
    """Zero-bubble interleaved schedule (reference pipeline_zero_bubble.py ZBVPP): the VPP job order with each
    virtual step's weight gradients as a separate backward_w job (parallel/pp_schedules.py zbvpp; executed by
    parallel/pipeline.py PipelineParallelZeroBubbleVPP)."""
    _mode = "ZBVPP"

    def _create_job_list(self):
        n, s, d = (int(self.get_attr(k)) for k in ("num_micro_batches", "pp_stage", "pp_degree"))
        v = int(self.get_attr("vpp_degree", 1))
        jobs = [Job(_KIND[k], PS.vpp_mb(i, d, v), PS.vpp_chunk(i, d, v, k == "F")) for k, i in PS.zbvpp(d, s, n, v)]
        jobs.append(Job(OPT))
        return jobs


def job_pairs(jobs):
    """("F" | "B" | "W", micro-batch) pairs of a job list, the optimizer job dropped."""
    return [j.as_tuple() for j in jobs if j.type() != OPT]
