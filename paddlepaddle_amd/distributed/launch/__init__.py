"""paddle.distributed.launch — start one worker process per GPU and supervise them.

Reference: python/paddle/distributed/launch/ (main.py, controllers/collective.py, job/, watcher).
Usage: ``python -m paddlepaddle_amd.distributed.launch --nproc_per_node 8 train.py --args``
(or ``--devices 0,1,2,3``). Per worker: HIP_VISIBLE_DEVICES-free device binding via LOCAL_RANK,
torch.distributed env (RANK/WORLD_SIZE/MASTER_*), PADDLE_* env, log file ``{log_dir}/workerlog.{rank}``.
Failure detection: the supervisor polls the workers; when one exits non-zero it terminates the rest
(their process groups), reports which rank failed with the tail of its log, and exits with that code —
optionally restarting the whole job up to ``--max_restart`` times.

Parameter-server mode (reference launch/controllers/ps.py): ``--server_num S --trainer_num T`` (or
``--servers ip:port,... --trainers ip:port,...``) starts S server and T trainer processes with the PS
environment (TRAINING_ROLE, PADDLE_PSERVERS_IP_PORT_LIST, PADDLE_TRAINERS_NUM, PADDLE_TRAINER_ID, POD_IP,
PADDLE_PORT); logs ``serverlog.i`` / ``workerlog.i``; the job ends when every trainer has exited.

Elastic mode (reference launch/controllers/master.py ETCDMaster + distributed/elastic.py): with
``--elastic_server host:port`` the desired worker count lives in a key-value store at that endpoint
(a c10d TCPStore, hosted by the node-0 launcher; etcd is not needed) under ``/paddle/<job_id>/np``.
``python -m paddlepaddle_amd.distributed.elastic --elastic_server ... --job_id ... --np N scale`` changes
it; the launcher then stops the workers and restarts them with the new world size (bounded by
``--np MIN:MAX`` and the local devices). Worker failures restart the job when ``--elastic_level 1``
(up to ``--max_restart`` times).
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
    # parameter server
    p.add_argument("--servers", default="", help="server endpoints (ip:port,...)")
    p.add_argument("--trainers", default="", help="trainer endpoints (ip:port,...)")
    p.add_argument("--server_num", type=int, default=None)
    p.add_argument("--trainer_num", type=int, default=None)
    # elastic
    p.add_argument("--elastic_server", default=None, help="host:port of the elastic key-value store")
    p.add_argument("--np", default=None, help="worker count MIN or MIN:MAX (elastic)")
    p.add_argument("--elastic_level", type=int, default=-1)
    p.add_argument("--elastic_timeout", type=int, default=30)
    # auto tuner (reference launch/main.py --auto_tuner_json): search the parallel configuration by trials
    p.add_argument("--auto_tuner_json", default=None, help="auto tuner config (json): run trials, keep the best")
    p.add_argument("--max_time_per_task", type=float, default=None, help="seconds before a job is stopped")
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
    if a.auto_tuner_json:
        return _launch_auto_tuner(a)
    if a.run_mode == "ps" or a.server_num or a.servers:
        return _launch_ps(a)
    if a.elastic_server:
        return _launch_elastic(a)
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


def _spawn(a, devs, world, host, port, node_rank=0, tag="workerlog"):
    local = len(devs)
    procs = []
    for i, d in enumerate(devs):
        rank = node_rank * local + i
        env = dict(os.environ)
        env.update(MASTER_ADDR=host, MASTER_PORT=port, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(i),
                   LOCAL_WORLD_SIZE=str(local), PADDLE_TRAINER_ID=str(rank), PADDLE_TRAINERS_NUM=str(world),
                   PADDLE_LOCAL_RANK=str(i), PADDLE_RANK_IN_NODE=str(i), PADDLE_LOCAL_DEVICE_IDS=d,
                   PADDLE_WORLD_DEVICE_IDS=",".join(devs), PADDLE_JOB_ID=a.job_id,
                   PADDLE_MASTER=f"{host}:{port}", HSA_ENABLE_IPC_MODE_LEGACY="0", PADDLE_AMD_DEVICE_ID=d)
        log = open(os.path.join(a.log_dir, f"{tag}.{rank}"), "w")
        cmd = [sys.executable, "-u", a.training_script] + list(a.training_script_args)
        p = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
        procs.append((rank, p, log))
    return procs


def _launch_ps(a):
    """Servers + trainers of a parameter-server job on this node."""
    servers = [e for e in a.servers.split(",") if e]
    trainers = [e for e in a.trainers.split(",") if e]
    if not servers:
        servers = [f"127.0.0.1:{_free_port()}" for _ in range(a.server_num or 1)]
    n_tr = len(trainers) or a.trainer_num or a.nproc_per_node or 1
    if not trainers:
        trainers = [f"127.0.0.1:{_free_port()}" for _ in range(n_tr)]
    os.makedirs(a.log_dir, exist_ok=True)
    base = dict(os.environ)
    base.update(PADDLE_PSERVERS_IP_PORT_LIST=",".join(servers), PADDLE_TRAINER_ENDPOINTS=",".join(trainers),
                PADDLE_TRAINERS_NUM=str(n_tr), PADDLE_JOB_ID=a.job_id, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs, trainer_pids = [], set()
    for role, eps in (("PSERVER", servers), ("TRAINER", trainers)):
        for i, ep in enumerate(eps):
            ip, port = ep.rsplit(":", 1)
            env = dict(base)
            env.update(TRAINING_ROLE=role, POD_IP=ip, PADDLE_PORT=port, PADDLE_TRAINER_ID=str(i),
                       PADDLE_CURRENT_ENDPOINT=ep)
            if role == "TRAINER":
                env.update(LOCAL_RANK=str(i), PADDLE_LOCAL_RANK=str(i))
            tag = "serverlog" if role == "PSERVER" else "workerlog"
            log = open(os.path.join(a.log_dir, f"{tag}.{i}"), "w")
            cmd = [sys.executable, "-u", a.training_script] + list(a.training_script_args)
            p = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
            procs.append((f"{role.lower()}{i}", p, log))
            if role == "TRAINER":
                trainer_pids.add(p.pid)
    try:
        while True:
            for name, p, log in procs:
                rc = p.poll()
                if rc is not None and rc != 0:
                    log.flush()
                    print(f"[launch] {name} exited with code {rc}; stopping the job.\n{_tail(log.name)}",
                          file=sys.stderr)
                    _terminate(procs)
                    return rc
            if all(p.poll() == 0 for _, p, _ in procs if p.pid in trainer_pids):
                deadline = time.time() + 60  # servers leave run_server once every trainer stopped
                while any(p.poll() is None for _, p, _ in procs) and time.time() < deadline:
                    time.sleep(a.poll_interval)
                _terminate(procs)
                return 0
            time.sleep(a.poll_interval)
    except KeyboardInterrupt:
        _terminate(procs)
        return 130
    finally:
        for _, _, log in procs:
            log.close()


def _np_range(a, ndev):
    if a.np is None:
        return ndev, ndev
    lo, _, hi = str(a.np).partition(":")
    return int(lo), int(hi or lo)


def _launch_elastic(a):
    """Single-node elastic job: restart the workers with a new world size whenever the store's np changes."""
    from ..elastic import Command
    devs_all = _devices(a)
    lo, hi = _np_range(a, len(devs_all))
    hi = min(hi, len(devs_all))
    cmd = Command(a.elastic_server, a.job_id, host=a.node_rank == 0)
    want = cmd.get_np()
    if want is None:
        cmd.set_np(lo if a.np is not None else len(devs_all))
        want = cmd.get_np()
    os.makedirs(a.log_dir, exist_ok=True)
    restarts = 0
    try:
        while True:
            n = max(lo, min(hi, want))
            host, port = "127.0.0.1", str(_free_port())
            print(f"[launch] elastic: starting {n} worker(s)", file=sys.stderr)
            procs = _spawn(a, devs_all[:n], n, host, port)
            rc, changed = _watch_elastic(procs, a, cmd, want)
            if changed is not None:
                want = changed
                continue
            if rc == 0:
                return 0
            if a.elastic_level < 1 or restarts >= a.max_restart:
                return rc
            restarts += 1
            print(f"[launch] elastic: restarting after failure ({restarts}/{a.max_restart})", file=sys.stderr)
    finally:
        cmd.close()


def _watch_elastic(procs, a, cmd, want):
    try:
        while True:
            alive = 0
            for rank, p, log in procs:
                rc = p.poll()
                if rc is None:
                    alive += 1
                elif rc != 0:
                    log.flush()
                    print(f"[launch] worker rank {rank} exited with code {rc}.\n{_tail(log.name)}", file=sys.stderr)
                    _terminate(procs)
                    return rc, None
            if alive == 0:
                return 0, None
            now = cmd.get_np()
            if now is not None and now != want:
                print(f"[launch] elastic: np {want} -> {now}; restarting the workers", file=sys.stderr)
                _terminate(procs)
                return None, now
            time.sleep(a.poll_interval)
    finally:
        for _, _, log in procs:
            log.close()


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


def _launch_auto_tuner(a):
    """Trial loop of the auto tuner (distributed/auto_tuner): each configuration runs as an ordinary collective
    job (its own log dir ``<log_dir>/trial_<k>``, the config as ``PADDLE_AUTO_TUNER_CFG`` json in the workers'
    environment and as script flags through the tuner's ``run_cmd``), the metric is read from rank 0's log,
    failures / out-of-memory runs are recorded as such (and prune the configs they dominate), ``history.csv``
    is rewritten after every trial and ``best_cfg.json`` names the winner."""
    import json
    from ..auto_tuner import AutoTuner, HistoryRecorder, gen_new_args, parse_metric
    with open(a.auto_tuner_json) as f:
        cfg = json.load(f)
    devs = _devices(a)
    cfg.setdefault("num_gpus", len(devs) * int(str(a.nnodes).split(":")[0]))
    cfg.setdefault("gpus_per_node", len(devs))
    tuner, rec = AutoTuner(cfg), HistoryRecorder(cfg)
    metric = cfg.setdefault("metric_cfg", {"name": "tokens/s", "OptimizationDirection": "Maximize"})
    per_task = a.max_time_per_task or cfg.get("max_time_per_task")
    base = a.log_dir
    os.makedirs(base, exist_ok=True)
    job = 0
    while True:
        c = tuner.search_once()
        if c is None:
            break
        job += 1
        trial_dir = os.path.join(base, f"trial_{job}")
        argv = ["--devices", ",".join(devs), "--log_dir", trial_dir, "--job_id", f"{a.job_id}_t{job}"]
        if per_task:
            argv += ["--max_time_per_task", str(per_task)]
        argv += [a.training_script] + gen_new_args(a.training_script_args, c, cfg)
        os.environ["PADDLE_AUTO_TUNER_CFG"] = json.dumps(c)
        print(f"[auto_tuner] trial {job}: {c}", file=sys.stderr)
        t0 = time.time()
        rc = launch(argv)
        os.environ.pop("PADDLE_AUTO_TUNER_CFG", None)
        text = ""
        try:
            with open(os.path.join(trial_dir, "workerlog.0"), errors="replace") as f:
                text = f.read()
        except OSError:
            pass
        value = parse_metric(text, metric)
        low = text.lower()
        entry = dict(c, job_id=job, time=round(time.time() - t0, 1), exit_code=rc)
        entry[metric["name"]] = value
        entry["oom"] = "out of memory" in low or "outofmemory" in low
        entry["error"] = rc != 0 or value is None
        rec.add_cfg(**entry)
        tuner.add_cfg(entry)
        rec.store_history(os.path.join(base, "history.csv"))
    best, none = rec.get_best()
    if none:
        print("[auto_tuner] no trial produced the metric", file=sys.stderr)
        return 1
    with open(os.path.join(base, "best_cfg.json"), "w") as f:
        json.dump(best, f, indent=1, default=str)
    print(f"[auto_tuner] best of {job} trials: {best}", file=sys.stderr)
    return 0


def _watch(procs, a):
    deadline = time.time() + a.max_time_per_task if getattr(a, "max_time_per_task", None) else None
    try:
        while True:
            if deadline is not None and time.time() > deadline:
                print(f"[launch] job exceeded --max_time_per_task ({a.max_time_per_task} s); stopping it.",
                      file=sys.stderr)
                _terminate(procs)
                return 124
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
