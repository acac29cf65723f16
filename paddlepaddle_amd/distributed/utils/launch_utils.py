"""Launch helpers. Reference: python/paddle/distributed/utils/launch_utils.py (find_free_ports, get_host_name_ip,
terminate_local_procs, get_gpus, add_arguments). The launcher itself is paddle.distributed.launch."""
from __future__ import annotations

import os
import signal
import socket
import time


def get_host_name_ip():
    try:
        name = socket.gethostname()
        return name, socket.gethostbyname(name)
    except OSError:
        return None


def find_free_ports(num):
    ports, socks = set(), []
    while len(ports) < num:
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        s.bind(("127.0.0.1", 0))
        ports.add(s.getsockname()[1])
        socks.append(s)
    for s in socks:
        s.close()
    return ports


def get_gpus(selected_gpus):
    import torch
    if selected_gpus is None:
        return list(range(torch.cuda.device_count()))
    return [int(x) for x in str(selected_gpus).split(",") if x.strip() != ""]


def add_arguments(argname, type, default, help, argparser, **kwargs):
    type = (lambda v: str(v).lower() in ("true", "1", "yes")) if type is bool else type
    argparser.add_argument("--" + argname, default=default, type=type, help=help + " Default: %(default)s.",
                           **kwargs)


def terminate_local_procs(procs):
    for p in procs:
        proc = getattr(p, "proc", p)
        if proc.poll() is None:
            proc.terminate()
    deadline = time.time() + 5
    for p in procs:
        proc = getattr(p, "proc", p)
        while proc.poll() is None and time.time() < deadline:
            time.sleep(0.1)
        if proc.poll() is None:
            os.kill(proc.pid, signal.SIGKILL)
