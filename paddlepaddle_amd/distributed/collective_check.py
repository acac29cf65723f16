"""Cross-rank collective-sequence checker (debug mode).

Reference: paddle/phi/core/distributed/comm_task_manager.cc:137 (the comm task manager tracks every collective per
communicator; FLAGS_enable_async_trace dumps per-rank sequences to find the rank that diverged) and
comm_task.h (op type, group, numel, dtype per task).

RCCL matches collectives by issue order alone: if one rank issues its bucket all-reduces, sharding
all-gathers / reduce-scatters or pipeline sends in a different order (or with a different shape) than its peers,
the job hangs or silently reduces the wrong buffers. With the checker on, every torch.distributed call made by
this framework (DataParallel buckets, the sharding engine, pipeline p2p, the paddle.distributed API) is
fingerprinted per communicator — (op, shapes, dtypes, reduce op) in issue order, folded into a running digest —
and ``check_collectives()`` compares the digests of all members of every group over a private gloo group at the
end of a step (DataParallel backward, the sharding engine step, pipeline train_batch call it automatically),
raising on the first divergence with both ranks' recent entries. Point-to-point traffic is checked per direction:
rank a's sends to b must equal b's receives from a.

Enable: ``PADDLE_AMD_CHECK_COLLECTIVES=1`` at init_parallel_env, or ``enable_collective_check()``.

Flight recorder (a hang never reaches the end-of-step check): with ``PADDLE_AMD_COLLECTIVE_TRACE_DIR`` set (or
``enable_collective_check(trace_dir=...)``) every fingerprint is also appended, flushed, to
``<dir>/collectives.rank<r>.log`` as it is issued (``<communicator> #<n> <entry>``), so after a hang or a kill the
per-rank files show where each rank stopped; ``first_divergence(paths)`` / ``tools/collective_trace_diff.py`` name
the first communicator entry at which two ranks disagree, or the ranks that stopped short.
"""
from __future__ import annotations

import contextlib
import functools
import hashlib
import os
import threading

import torch
import torch.distributed as dist

_OPS = ("all_reduce", "all_gather", "all_gather_into_tensor", "reduce_scatter_tensor", "reduce_scatter",
        "broadcast", "reduce", "all_to_all", "all_to_all_single", "send", "recv", "isend", "irecv", "barrier",
        "gather", "scatter")
_P2P_SEND = ("send", "isend")
_P2P_RECV = ("recv", "irecv")
_ORIG = {}
_STATE = {"on": False, "pg": None, "checks": 0}
_SEQ = {}      # key -> [count, hasher, recent entries]
_KEEP = 16     # entries kept per key for the divergence report
_TLS = threading.local()
_TRACE = {"f": None}


@contextlib.contextmanager
def label(text):
    """Name the collectives issued inside (e.g. "dp bucket 3", "rs unit 7"): the label is part of their
    fingerprint, so two ranks that issue same-shaped collectives for different buckets are caught too."""
    prev = getattr(_TLS, "label", None)
    _TLS.label = text
    try:
        yield
    finally:
        _TLS.label = prev


class CollectiveMismatchError(RuntimeError):
    """Ranks issued different collective sequences on a communicator."""


def enabled():
    return _STATE["on"]


def _ranks_of(group):
    if group is None:
        return tuple(range(dist.get_world_size()))
    try:
        return tuple(dist.get_process_group_ranks(group))
    except Exception:  # pragma: no cover
        return ("?",)


def _desc(a):
    if isinstance(a, torch.Tensor):
        return f"{tuple(a.shape)}:{str(a.dtype).replace('torch.', '')}"
    if isinstance(a, (list, tuple)) and a and all(isinstance(x, torch.Tensor) for x in a):
        return "[" + ",".join(_desc(x) for x in a) + "]"
    return None


def _record(key, entry):
    s = _SEQ.get(key)
    if s is None:
        s = _SEQ[key] = [0, hashlib.sha1(), []]
    s[0] += 1
    s[1].update(entry.encode())
    s[2].append(f"#{s[0]} {entry}")
    f = _TRACE["f"]
    if f is not None:
        f.write(f"{_key_str(key)} #{s[0]} {entry}\n")
        f.flush()
    if len(s[2]) > _KEEP:
        del s[2][0]


def _key_str(key):
    return f"{key[0]}:{'-'.join(str(r) for r in key[1])}" if key[0] == "coll" else f"p2p:{key[1]}>{key[2]}"


def _fingerprint(name, args, kwargs):
    group = kwargs.get("group")
    tensors = [d for d in (_desc(a) for a in list(args) + [v for k, v in kwargs.items() if k != "group"]) if d]
    op = kwargs.get("op")
    if op is None:
        for a in args:
            if isinstance(a, dist.ReduceOp) or type(a).__name__ in ("ReduceOp", "RedOpType"):
                op = a
    red = f" op={op}" if op is not None else ""
    lab = getattr(_TLS, "label", None)
    if lab:
        red += f" [{lab}]"
    me = dist.get_rank()
    if name in _P2P_SEND or name in _P2P_RECV:
        peer = kwargs.get("dst", kwargs.get("src"))
        if peer is None:
            ints = [a for a in args if isinstance(a, int)]
            peer = ints[0] if ints else -1
        a, b = (me, peer) if name in _P2P_SEND else (peer, me)
        return ("p2p", a, b), f"p2p {a}->{b} {' '.join(tensors)}{red}"
    return ("coll", _ranks_of(group)), f"{name} {' '.join(tensors)}{red}"


def _wrap(name, fn):
    @functools.wraps(fn)
    def w(*args, **kwargs):
        if _STATE["on"]:
            key, entry = _fingerprint(name, args, kwargs)
            _record(key, entry)
        return fn(*args, **kwargs)
    return w


def enable_collective_check(trace_dir=None):
    """Fingerprint every torch.distributed collective from here on (wraps whatever is installed: composes with
    the comm watchdog) and create the private gloo group the checks run on. ``trace_dir`` (default
    ``$PADDLE_AMD_COLLECTIVE_TRACE_DIR``): also append every fingerprint to this rank's flight-recorder file."""
    if not dist.is_initialized():
        raise RuntimeError("enable_collective_check: call init_parallel_env first")
    trace_dir = trace_dir or os.environ.get("PADDLE_AMD_COLLECTIVE_TRACE_DIR")
    if trace_dir and _TRACE["f"] is None:
        os.makedirs(trace_dir, exist_ok=True)
        _TRACE["f"] = open(os.path.join(trace_dir, f"collectives.rank{dist.get_rank()}.log"), "a", buffering=1)
    if _STATE["pg"] is None:
        _STATE["pg"] = dist.new_group(backend="gloo")  # collective over the world: every rank calls this
    if not _STATE.get("atexit"):
        import atexit
        import sys
        rank = dist.get_rank()

        def _report():
            if _STATE["on"] and _STATE["checks"]:
                sys.stderr.write(f"[collective-check] rank {rank}: {_STATE['checks']} cross-rank "
                                 f"sequence checks passed\n")
        atexit.register(_report)
        _STATE["atexit"] = True
    if not _ORIG:
        for n in _OPS:
            f = getattr(dist, n, None)
            if f is not None:
                _ORIG[n] = f
                setattr(dist, n, _wrap(n, f))
    _STATE["on"] = True


def disable_collective_check():
    _STATE["on"] = False
    if _TRACE["f"] is not None:
        _TRACE["f"].close()
        _TRACE["f"] = None
    for n, f in _ORIG.items():
        setattr(dist, n, f)
    _ORIG.clear()
    _SEQ.clear()


def local_sequences():
    """{key: (count, digest, recent entries)} of this rank (for tests / debugging)."""
    return {k: (v[0], v[1].hexdigest(), list(v[2])) for k, v in _SEQ.items()}


def check_collectives(where="step"):
    """Compare this step's collective sequences with every peer's (collective over the world: all ranks must
    call it at the same point). Raises CollectiveMismatchError naming the communicator, the ranks and their
    last entries on the first divergence; resets the sequences otherwise."""
    if not _STATE["on"]:
        return
    mine = local_sequences()
    gather = _ORIG.get("all_gather_object") or dist.all_gather_object
    world = dist.get_world_size()
    objs = [None] * world
    gather(objs, (dist.get_rank(), mine), group=_STATE["pg"])
    by_rank = dict(objs)
    _STATE["checks"] += 1
    problems = []
    keys = set()
    for r, seqs in by_rank.items():
        keys.update(seqs)
    for key in sorted(keys, key=repr):
        if key[0] == "coll":
            members = [r for r in key[1] if isinstance(r, int)]
            views = {r: by_rank.get(r, {}).get(key) for r in members}
        else:  # p2p a->b: a's send log vs b's receive log
            views = {r: by_rank.get(r, {}).get(key) for r in (key[1], key[2]) if isinstance(r, int) and 0 <= r < world}
        sigs = {r: (v[0], v[1]) if v is not None else (0, None) for r, v in views.items()}
        if len(set(sigs.values())) > 1:
            detail = "; ".join(f"rank {r}: {sigs[r][0]} ops, last {views[r][2][-3:] if views[r] else []}"
                               for r in sorted(views))
            problems.append(f"{key[0]} {key[1:]}: {detail}")
    _SEQ.clear()
    if problems:
        raise CollectiveMismatchError(f"collective sequences diverged at {where} (check #{_STATE['checks']}): "
                                      + " | ".join(problems))


def maybe_enable_from_env():
    if os.environ.get("PADDLE_AMD_CHECK_COLLECTIVES", "0") not in ("", "0", "false", "False"):
        enable_collective_check()


def first_divergence(paths):
    """Compare flight-recorder files (``collectives.rank<r>.log``, one per rank): for every communicator, the first
    entry index at which its members' logs differ, and members whose log ends earlier than their peers' (the ranks
    a hang left behind). Returns a list of human-readable findings (empty: the logs agree)."""
    import re
    logs = {}
    for p in paths:
        m = re.search(r"rank(\d+)", os.path.basename(p))
        r = int(m.group(1)) if m else len(logs)
        per = {}
        with open(p) as f:
            for line in f:
                k, _, rest = line.rstrip("\n").partition(" ")
                per.setdefault(k, []).append(rest.split(" ", 1)[1] if " " in rest else rest)
        logs[r] = per
    out = []
    keys = sorted({k for per in logs.values() for k in per})
    for k in keys:
        if k.startswith("coll:"):
            members = [int(x) for x in k[5:].split("-") if x.lstrip("-").isdigit()]
        else:
            a, b = k[4:].split(">")
            members = [int(a), int(b)]
        seqs = {r: logs.get(r, {}).get(k, []) for r in members if r in logs}
        if len(seqs) < 2:
            continue
        n = min(len(v) for v in seqs.values())
        for i in range(n):
            if len({v[i] for v in seqs.values()}) > 1:
                out.append(f"{k} entry #{i + 1}: " + "; ".join(f"rank {r}: {v[i]}" for r, v in sorted(seqs.items())))
                break
        else:
            longest = max(len(v) for v in seqs.values())
            short = [r for r, v in sorted(seqs.items()) if len(v) < longest]
            if short:
                out.append(f"{k}: ranks {short} stopped after {n} of {longest} entries (next expected: "
                           f"{next(v for v in seqs.values() if len(v) == longest)[n]})")
    return out
