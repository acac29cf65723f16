"""paddle.distributed.launch — start one worker process per GPU and supervise them.

Reference: python/paddle/distributed/launch/ (main.py, controllers/collective.py, job/, watcher).
Usage: ``python -m paddlepaddle_amd.distributed.launch --nproc_per_node 8 train.py --args``
(or ``--devices 0,1,2,3``). Per worker: HIP_VISIBLE_DEVICES-free device binding via LOCAL_RANK,
torch.distributed env (RANK/WORLD_SIZE/MASTER_*), PADDLE_* env, log file ``{log_dir}/workerlog.{rank}``.
Failure detection: the supervisor polls the workers; when one exits non-zero it terminates the rest
(their process groups), reports which rank failed with the tail of its log, and exits with that code —
optionally restarting the whole job up to ``--max_restart`` times (elastic-lite).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def parse_args(argv=None):
    p = argparse.ArgumentParser("paddlepaddle_amd.distributed.launch")
    p.add_argument("--nproc_per_node", type=int, default=None)
    p.add_argument("--devices", "--gpus", dest="devices", default=None)
    p.add_argument("--nnodes", type=str, default="1")
    p.add_argument("--rank", "--node_rank", dest="node_rank", type=int, default=0)
    p.add_argument("--master", default=None, help="ip:port of the rendezvous master")
    p.add_argument("--log_dir", default="log")
    p.add_argument("--run_mode", default="collective")
    p.add_argument("--job_id", default="default")
    p.add_argument("--max_restart", type=int, default=0)
    p.add_argument("--poll_interval", type=float, default=0.5)
    p.add_argument("training_script")
    p.add_argument("training_script_args", nargs=argparse.REMAINDER)
    return p.parse_args(argv)


def _devices(a):
    if a.devices:
        return [d for d in a.devices.split(",") if d != ""]
    n = a.nproc_per_node
    if n is None:
        try:
            import torch
            n = max(torch.cuda.device_count(), 1)
        except Exception:
            n = 1
    return [str(i) for i in range(n)]


def _tail(path, n=20):
    try:
        with open(path, "rb") as f:
            return b"".join(f.readlines()[-n:]).decode(errors="replace")
    except OSError:
        return ""


def launch(argv=None):
    a = parse_args(argv)
    devs = _devices(a)
    nnodes = int(str(a.nnodes).split(":")[0])
    local = len(devs)
    world = local * nnodes
    if a.master:
        host, port = a.master.split(":")
    else:
        host, port = "127.0.0.1", str(_free_port())
    os.makedirs(a.log_dir, exist_ok=True)
    attempt = 0
    while True:
        procs = []
        for i, d in enumerate(devs):
            rank = a.node_rank * local + i
            env = dict(os.environ)
            env.update(MASTER_ADDR=host, MASTER_PORT=port, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(i),
                       LOCAL_WORLD_SIZE=str(local), PADDLE_TRAINER_ID=str(rank), PADDLE_TRAINERS_NUM=str(world),
                       PADDLE_LOCAL_RANK=str(i), PADDLE_RANK_IN_NODE=str(i), PADDLE_LOCAL_DEVICE_IDS=d,
                       PADDLE_WORLD_DEVICE_IDS=",".join(devs), PADDLE_JOB_ID=a.job_id,
                       PADDLE_MASTER=f"{host}:{port}", HSA_ENABLE_IPC_MODE_LEGACY="0",
                       PADDLE_AMD_DEVICE_ID=d)
            log = open(os.path.join(a.log_dir, f"workerlog.{rank}"), "w")
            cmd = [sys.executable, "-u", a.training_script] + list(a.training_script_args)
            p = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
            procs.append((rank, p, log))
        rc = _watch(procs, a)
        if rc == 0 or attempt >= a.max_restart:
            return rc
        attempt += 1
        print(f"[launch] restarting job (attempt {attempt}/{a.max_restart})", file=sys.stderr)


def _terminate(procs):
    for _, p, _ in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except OSError:
                pass
    deadline = time.time() + 10
    for _, p, _ in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.1)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass


def _watch(procs, a):
    try:
        while True:
            alive = 0
            for rank, p, log in procs:
                rc = p.poll()
                if rc is None:
                    alive += 1
                elif rc != 0:
                    log.flush()
                    print(f"[launch] worker rank {rank} exited with code {rc}; stopping the job.\n"
                          f"--- tail of {a.log_dir}/workerlog.{rank} ---\n{_tail(log.name)}", file=sys.stderr)
                    _terminate(procs)
                    return rc
            if alive == 0:
                return 0
            time.sleep(a.poll_interval)
    except KeyboardInterrupt:
        _terminate(procs)
        return 130
    finally:
        for _, _, log in procs:
            log.close()


def main():
    sys.exit(launch())


if __name__ == "__main__":
    main()
