"""Tagged point-to-point messages between pipeline stages, with the meta exchanged once per shape.

Reference: python/paddle/distributed/fleet/meta_parallel/pp_utils/p2p_communication.py:52 (SendRecvMeta: the
tensor meta is sent once and cached), :656-670 (later sends skip the meta).

Design (MI355X): payloads are device tensors on the pipeline group's backend (RCCL over xGMI), sent with
non-blocking ``isend`` so a stage can run ahead of its neighbour. Routing needs a small tag per message
(which micro-batch / chunk / direction it is: the interleaved and zero-bubble schedules consume messages in a
different order than a neighbour produces them on a shared channel). The tag travels on a host-side twin of the
group (gloo): reading it costs the host a tiny TCP message, never a device -> host synchronisation, and the
device stream is only ever ordered by RCCL itself. The tensor meta (rank, shape, dtype) rides in the same tag
message only when it changes for that directed channel and message class (direction + slot / chunk); both ends
cache it, so a steady training run performs one meta exchange per (channel, message class, shape). Messages
that arrive ahead of the one asked for are stashed.

Ordered mode (``ordered=True``: 1F1B / FThenB / ZBH1 pipelines and the static engine, whose stages consume every
directed channel in the order the neighbour produces it — the schedule fixes the tag order): no per-message
header. Each end calls ``begin_run()`` at the start of a schedule run; the first message of each (channel,
class) in a run carries the meta on the host twin, every other payload receive is posted straight on RCCL with
the cached meta, so the receiving host never waits on a gloo message in the steady state. A shape change inside a
run raises. The interleaved (VPP) schedules, whose consumption order differs from the production order on a
channel, keep the tagged protocol with the stash. With the collective checker on
(distributed/collective_check.py) every payload is labelled with its tag, so an order mismatch between the two
ends of a channel is reported at the end of the step.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.int64: 3, torch.int32: 4, torch.bool: 5,
       torch.uint8: 6, torch.float64: 7}
_CODE = {v: k for k, v in _DT.items()}
_MAXD = 8
_HDR = 4 + 2 + _MAXD  # tag[3], meta flag, ndim, dtype, shape[8]


def host_twin(ranks_lists, my_rank):
    """Create gloo twins for every rank list (collective over the world: every rank calls this with the same
    lists in the same order); returns the twin containing ``my_rank`` (None for gloo worlds: the group itself
    already carries host tensors)."""
    if not dist.is_initialized() or dist.get_backend() == "gloo":
        return None
    mine = None
    for ranks in ranks_lists:
        if len(ranks) < 2:
            continue
        g = dist.new_group(ranks=sorted(ranks), backend="gloo")
        if my_rank in ranks:
            mine = g
    return mine


class P2P:
    """``send(t, dst, tag)`` / ``recv(src, tag)`` / ``join()``. ``group``: the payload process group (None =
    world); ``host_group``: its gloo twin (None when ``group`` is gloo already). Ranks are global ranks."""

    def __init__(self, dev, group=None, host_group=None, ordered=False):
        self.dev = dev
        self.pg = group
        self.hpg = host_group if host_group is not None else group
        self.ordered = ordered
        self.pending = []
        self.stash = {}
        self.sent_meta = {}
        self.recv_meta = {}
        self.meta_exchanges = 0   # sends that carried a new meta (one per channel and shape in a steady run)
        self.messages = 0
        self.headers = 0          # host-side header messages sent (ordered mode: first of each class per run)
        self._run_sent = set()
        self._run_recv = set()

    def begin_run(self):
        """Start of a schedule run (ordered mode): the first message of each (channel, class) carries the meta."""
        self._run_sent.clear()
        self._run_recv.clear()

    def _label(self, tag):
        from ..distributed import collective_check as _cc
        import contextlib
        return _cc.label(f"p2p tag {tuple(int(v) for v in tag)}") if _cc.enabled() else contextlib.nullcontext()

    def _header(self, tag, new, t):
        hdr = [int(tag[0]), int(tag[1]), int(tag[2]), int(new), t.dim(), _DT[t.dtype]]
        hdr += list(t.shape) + [0] * (_MAXD - t.dim())
        h = torch.tensor(hdr, dtype=torch.int64)
        if self.hpg is self.pg and t.device.type != "cpu":  # a device-only group: the tag travels as a device tensor
            h = h.to(t.device)
        return h

    def send(self, t, dst, tag):
        t = t.contiguous()
        if t.dim() > _MAXD:
            raise ValueError(f"pipeline p2p supports tensors of up to {_MAXD} dims, got {t.dim()}")
        meta = (tuple(t.shape), t.dtype)
        key = (dst, int(tag[0]), int(tag[1]))  # channel + message class (direction, slot / chunk); not the mb
        new = self.sent_meta.get(key) != meta
        if self.ordered:
            if key in self._run_sent:
                if new:
                    raise RuntimeError(f"pipeline p2p (ordered): message {tuple(tag)} to rank {dst} changed shape "
                                       f"within a run ({self.sent_meta[key]} -> {meta})")
            else:  # first of its class this run: the header carries the meta
                self._run_sent.add(key)
                self.sent_meta[key] = meta
                self.meta_exchanges += int(new)
                h = self._header(tag, 1, t)
                self.pending.append((dist.isend(h, dst, group=self.hpg), h))
                self.headers += 1
            with self._label(tag):
                self.pending.append((dist.isend(t, dst, group=self.pg), t))
            self.messages += 1
            return
        if new:
            self.sent_meta[key] = meta
            self.meta_exchanges += 1
        h = self._header(tag, new, t)
        self.pending.append((dist.isend(h, dst, group=self.hpg), h))
        self.headers += 1
        with self._label(tag):
            self.pending.append((dist.isend(t, dst, group=self.pg), t))
        self.messages += 1

    def recv(self, src, tag):
        if self.ordered:
            key = (src, int(tag[0]), int(tag[1]))
            if key not in self._run_recv:
                h = torch.empty(_HDR, dtype=torch.int64,
                                device=self.dev if (self.hpg is self.pg and self.dev.type != "cpu") else "cpu")
                dist.recv(h, src, group=self.hpg)
                v = h.tolist()
                if (v[0], v[1]) != key[1:]:
                    raise RuntimeError(f"pipeline p2p (ordered): expected class {key[1:]} from rank {src}, the "
                                       f"neighbour sent {(v[0], v[1])} first: its schedule disagrees with this one")
                self.recv_meta[key] = (tuple(v[6:6 + v[4]]), _CODE[v[5]])
                self._run_recv.add(key)
            shape, dt = self.recv_meta[key]
            t = torch.empty(shape, dtype=dt, device=self.dev)
            with self._label(tag):
                dist.recv(t, src, group=self.pg)
            return t
        st = self.stash.setdefault(src, {})
        want = tuple(int(v) for v in tag)
        if want in st:
            return st.pop(want)
        dev_hdr = self.hpg is self.pg and self.dev.type != "cpu"
        while True:
            h = torch.empty(_HDR, dtype=torch.int64, device=self.dev if dev_hdr else "cpu")
            dist.recv(h, src, group=self.hpg)
            v = h.tolist()
            key = (src, v[0], v[1])
            if v[3]:
                self.recv_meta[key] = (tuple(v[6:6 + v[4]]), _CODE[v[5]])
            shape, dt = self.recv_meta[key]
            t = torch.empty(shape, dtype=dt, device=self.dev)
            with self._label(v[:3]):
                dist.recv(t, src, group=self.pg)
            got = (v[0], v[1], v[2])
            if got == want:
                return t
            st[got] = t

    def join(self):
        for w, _ in self.pending:
            w.wait()
        self.pending = []
