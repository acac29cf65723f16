"""Native collective watchdog (CommTaskManager equivalent): host-task timeout reporting, and a 2-rank gloo
job where one rank enters an all_reduce late — the other rank's watchdog must report the pending
all_reduce with its group and size, and the job must still complete."""
import os
import sys
import time

import numpy as np
import pytest
import torch

from test_distributed_cpu import ROOT, _setup, _spawn


def _wd():
    sys.path.insert(0, ROOT)
    from paddlepaddle_amd.utils import native
    m = native.module()
    if m is None or not hasattr(m, "comm_watchdog"):
        pytest.skip("native runtime not built")
    return m.comm_watchdog


def test_host_task_timeout_reported(tmp_path):
    wd = _wd()
    wd.start(0, 200, 50, False, str(tmp_path))
    t0 = wd.timeouts()
    a = wd.track_host("all_reduce", "world", 4096, 0)
    b = wd.track_host("broadcast", "world", 16, 10_000)
    time.sleep(0.6)
    assert wd.timeouts() == t0 + 1
    assert "all_reduce" in wd.timed_out_ops()
    wd.finish(a)
    wd.finish(b)
    assert wd.pending() == 0
    rep = (tmp_path / "comm_watchdog.rank0.txt").read_text()
    assert "op=all_reduce" in rep and "bytes=4096" in rep
    wd.stop()


def _late_worker(rank, world, port, tmpdir, q):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.distributed import watchdog
    paddle.distributed.enable_comm_watchdog(timeout_s=0.3, poll_ms=50, report_dir=tmpdir)
    t = paddle.to_tensor(np.ones(8, dtype="float32") * (rank + 1))
    if rank == 1:
        time.sleep(1.5)
    paddle.distributed.all_reduce(t)
    st = watchdog.status()
    paddle.distributed.disable_comm_watchdog()
    q.put((rank, float(t.numpy()[0]), st))
    paddle.distributed.barrier()


def test_late_rank_detected_by_watchdog(tmp_path):
    res = dict((r, (v, st)) for r, v, st in _spawn(_late_worker, str(tmp_path)))
    assert res[0][0] == 3.0 and res[1][0] == 3.0
    pending, timeouts, ops = res[0][1]
    assert timeouts >= 1 and "all_reduce" in ops
    rep = (tmp_path / "comm_watchdog.rank0.txt").read_text()
    assert "op=all_reduce" in rep and "group=world" in rep


@pytest.mark.gpu
def test_device_task_retired_by_event():
    wd = _wd()
    wd.start(0, 60_000, 20, False, "")
    assert wd.device_events(), "hipEvent* not resolved from the loaded HIP runtime"
    a = torch.randn(4096, 4096, device="cuda")
    for _ in range(20):
        a = a @ a
        a = a / a.norm()
    tid = wd.track("all_reduce", "world", a.numel() * 4, torch.cuda.current_stream().cuda_stream, 0)
    assert tid > 0
    torch.cuda.synchronize()
    deadline = time.time() + 5
    while wd.pending() and time.time() < deadline:
        time.sleep(0.05)
    assert wd.pending() == 0
    wd.stop()
