"""Pipeline p2p under RCCL's rendezvous semantics, without hardware (parallel/pp_comm.py).

gloo buffers sends, so every CPU pipeline test passes even with a protocol that hangs on RCCL (a send completes
only while the matching receive is posted; a rank pair's ops run in issue order on one stream per communicator).
These tests replay the exact p2p programs the pipeline engines issue — batched send/recv groups per job, one
payload communicator per direction, eager headers with host-blocking reads — for every schedule and size, and
check that (a) none can deadlock, (b) the previous protocol (ungrouped isend + recv on one communicator) does,
(c) a deliberately reordered schedule is caught, and (d) the real engine issues exactly the modelled program.
Reference: pp_utils/p2p_communication.py:286 / :573 (batch_isend_irecv)."""
import os
import sys

import numpy as np
import pytest
import torch

from paddlepaddle_amd.parallel import pp_comm as C


@pytest.mark.parametrize("host_waits", [False, True])  # RCCL (stream waits) and gloo (host waits) semantics
@pytest.mark.parametrize("mode", ["1F1B", "FThenB", "Eager1F1B", "ZBH1"])
def test_schedules_cannot_deadlock(mode, host_waits):
    n = 0
    for S in range(2, 9):
        for M in range(1, 17):
            n += C.simulate(C.programs(mode, S, M), host_waits=host_waits)
    assert n > 0


@pytest.mark.parametrize("mode", ["VPP", "ZBVPP"])
@pytest.mark.parametrize("host_waits", [False, True])
def test_interleaved_schedule_cannot_deadlock(host_waits, mode):
    for S in range(2, 9):
        for V in (2, 3, 4):
            for M in range(S, 17, S):
                C.simulate(C.programs(mode, S, M, V), host_waits=host_waits)


def test_zbvpp_jobs_valid():
    from paddlepaddle_amd.parallel import pp_schedules as PS
    for S in range(2, 6):
        for V in (2, 3):
            for M in range(S, 13, S):
                for s in range(S):
                    jobs = PS.zbvpp(S, s, M, V)
                    base = PS.vpp(S, s, M, V)
                    assert [j for j in jobs if j[0] != "W"] == base  # the VPP order with W jobs inserted
                    PS.check(jobs, M * V, split_w=True)


@pytest.mark.parametrize("mode", ["1F1B", "Eager1F1B", "ZBH1"])
def test_previous_protocol_deadlocks(mode):
    """Ungrouped isend at the end of a job + separate receive, one communicator: the 1F1B steady state (stage s
    sends activation k then waits for gradient j; stage s + 1 sends gradient j then waits for activation k)."""
    hung = []
    for S in range(2, 9):
        for M in range(1, 17):
            try:
                C.simulate(C.programs(mode, S, M, batched=False, split_directions=False), per_direction=False)
            except C.Deadlock:
                hung.append((S, M))
    assert (4, 8) in hung and len(hung) > 50, hung


def test_single_communicator_interleaved_two_stages_deadlocks_without_direction_split():
    """At two stages the interleaved ring sends both ways on one pair: batching alone is not enough there."""
    with pytest.raises(C.Deadlock):
        C.simulate(C.programs("VPP", 2, 4, 2, split_directions=False), per_direction=False)


def test_reordered_schedule_is_caught():
    progs = C.programs("1F1B", 4, 8)
    st = progs[2]
    recv_groups = [i for i, g in enumerate(st) if any(op[0] == "r" and op[3][2][0] == "F" for op in g)]
    i, j = recv_groups[1], recv_groups[2]
    st[i], st[j] = st[j], st[i]  # stage 2 consumes two forward activations out of order
    with pytest.raises(C.Deadlock):
        C.simulate(progs)


# ---- the real engine issues the modelled program (2 gloo ranks)
sys.path.insert(0, os.path.dirname(__file__))


def _rec_worker(rank, world, port, schedule, acc, q):
    from test_distributed_cpu import _setup
    from test_fleet_cpu import _fleet_init, _mlp_descs, _mse, _pp_data
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.parallel.pipeline import PipelineLayer
    fleet = _fleet_init(paddle, acc=acc, pp_degree=2, schedule=schedule)
    vpp = schedule in ("VPP", "ZBVPP")
    pl = PipelineLayer(_mlp_descs(paddle), num_stages=2, loss_fn=_mse,
                       num_virtual_pipeline_stages=2 if vpp else None)
    opt = paddle.optimizer.SGD(1e-2, parameters=pl.parameters())
    model = fleet.distributed_model(pl)
    model._p2p_record = True
    opt = fleet.distributed_optimizer(opt)
    x, y = _pp_data()
    x, y = torch.cat([x] * (acc // 2)), torch.cat([y] * (acc // 2))
    model.train_batch([paddle.Tensor(x), paddle.Tensor(y)], opt)
    log = [tuple((k, int(peer), tuple(tg)) for k, peer, tg in g) for g in model._p2p.log]
    q.put((rank, log))
    paddle.distributed.barrier()


def _key(k):
    kind = {"F": 0, "B": 1}[k[0]]
    return (kind, int(k[1]), int(k[2]))


@pytest.mark.parametrize("schedule,acc", [("1F1B", 4), ("ZBH1", 4), ("Eager1F1B", 4), ("FThenB", 2), ("VPP", 4),
                                          ("ZBVPP", 4)])
def test_engine_issues_modelled_program(schedule, acc):
    from test_distributed_cpu import _spawn
    res = dict(_spawn(_rec_worker, schedule, acc, world=2))
    progs = C.programs(schedule, 2, acc, V=2 if schedule in ("VPP", "ZBVPP") else 1)
    for rank in (0, 1):
        want = [tuple((op[0], op[2] if op[0] == "s" else op[1], _key(op[3][2])) for op in g) for g in progs[rank]]
        assert res[rank] == want, (rank, res[rank], want)
