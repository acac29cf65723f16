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

Grouped payloads (reference p2p_communication.py:286 / :573 batch_isend_irecv): a payload send is queued, not
issued; the next payload receive issues the queued sends and itself as ONE batched p2p group (ncclGroupStart /
End), and a schedule job that receives nothing calls ``flush()`` first. RCCL / NCCL send / recv are rendezvous
operations on one stream per rank pair: an ungrouped ``isend`` followed by a ``recv`` deadlocks when the
neighbour does the same in the other direction (the 1F1B steady state: stage s sends activation k and waits for
gradient j while stage s + 1 sends gradient j and waits for activation k). Grouped, both directions progress in
one launch. parallel/pp_comm.py derives the per-stage op programs of every schedule and replays them under
rendezvous semantics (tests/test_pp_rendezvous.py); ``record=True`` logs the issued groups so a run of the real
engine can be compared with its program. Headers (host twin, gloo) stay eager: the receiver's host reads one
before it posts the payload receive. Payloads travel on two communicators by direction (to a higher global rank:
the pipe group; to a lower one: its twin, ``payload_twin``), so one RCCL stream never holds both a rank pair's
sends and its receives; a batched group is issued as one batch per direction, sends' directions first. With both
rules the replay finds no deadlock for any schedule (1F1B / FThenB / Eager1F1B / ZBH1 / interleaved, 2-8 stages,
1-16 micro-batches), the interleaved schedule at two stages included (its ring sends both ways on one pair).
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
    lists in the same order); returns the twin containing ``my_rank``. Gloo worlds get a twin too: headers then
    never share a FIFO channel with payloads (a payload queued before a later header would otherwise arrive after
    it), so the CPU runs exercise the same protocol as RCCL ones."""
    if not dist.is_initialized():
        return None
    mine = None
    for ranks in ranks_lists:
        if len(ranks) < 2:
            continue
        g = dist.new_group(ranks=sorted(ranks), backend="gloo")
        if my_rank in ranks:
            mine = g
    return mine


def payload_twin(ranks_lists, my_rank):
    """A second payload group for every rank list (default backend: RCCL on GPU, gloo on CPU; collective over the
    world: every rank calls this with the same lists in the same order); returns the one containing ``my_rank``.
    P2P sends messages from a lower to a higher global rank on the pipe group and the other direction on this twin,
    so no RCCL stream ever carries sends and receives of one rank pair (see parallel/pp_comm.py)."""
    if not dist.is_initialized():
        return None
    mine = None
    for ranks in ranks_lists:
        if len(ranks) < 2:
            continue
        g = dist.new_group(ranks=sorted(ranks))
        if my_rank in ranks:
            mine = g
    return mine


class P2P:
    """``send(t, dst, tag)`` / ``recv(src, tag)`` / ``join()``. ``group``: the payload process group (None =
    world); ``host_group``: its gloo twin (None when ``group`` is gloo already). Ranks are global ranks."""

    def __init__(self, dev, group=None, host_group=None, ordered=False, record=False, down_group=None):
        self.dev = dev
        self.pg = group
        self.pg_down = down_group if down_group is not None else group  # messages to a lower global rank
        self.hpg = host_group if host_group is not None else group
        self.ordered = ordered
        self.pending = []
        self.queued = []          # payload sends waiting for the next receive / flush (one batched group)
        self.record = record
        self.log = []             # record=True: issued groups, each a tuple of ("s" | "r", peer, tag)
        self.groups = 0           # batched groups issued
        self.stash = {}
        self.sent_meta = {}
        self.recv_meta = {}
        self.meta_exchanges = 0   # sends that carried a new meta (one per channel and shape in a steady run)
        self.messages = 0
        self.headers = 0          # host-side header messages sent (ordered mode: first of each class per run)
        self._run_sent = set()
        self._run_recv = set()
        # batch_isend_irecv on RCCL needs each group's communicator created by all of its ranks first: one tiny
        # all-reduce per payload group (every member builds its endpoint at the same point of the run)
        if dist.is_initialized() and dev is not None and getattr(dev, "type", "cpu") != "cpu":
            for g in {id(x): x for x in (self.pg, self.pg_down)}.values():
                dist.all_reduce(torch.zeros(1, device=dev), group=g)

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
            self.queued.append((t, dst, tuple(int(v) for v in tag)))
            self.messages += 1
            return
        if new:
            self.sent_meta[key] = meta
            self.meta_exchanges += 1
        h = self._header(tag, new, t)
        self.pending.append((dist.isend(h, dst, group=self.hpg), h))
        self.headers += 1
        self.queued.append((t, dst, tuple(int(v) for v in tag)))
        self.messages += 1

    def recv(self, src, tag):
        if self.ordered:
            key = (src, int(tag[0]), int(tag[1]))
            if key not in self._run_recv:
                self._issue(None)  # never hold queued sends while the host blocks on a header
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
            self._issue((t, src, tuple(int(v) for v in tag)))
            return t
        st = self.stash.setdefault(src, {})
        want = tuple(int(v) for v in tag)
        if want in st:
            return st.pop(want)
        dev_hdr = self.hpg is self.pg and self.dev.type != "cpu"
        self._issue(None)  # tagged mode: every message has a header the host blocks on; send the queued ones first
        while True:
            h = torch.empty(_HDR, dtype=torch.int64, device=self.dev if dev_hdr else "cpu")
            dist.recv(h, src, group=self.hpg)
            v = h.tolist()
            key = (src, v[0], v[1])
            if v[3]:
                self.recv_meta[key] = (tuple(v[6:6 + v[4]]), _CODE[v[5]])
            shape, dt = self.recv_meta[key]
            t = torch.empty(shape, dtype=dt, device=self.dev)
            got = (v[0], v[1], v[2])
            self._issue((t, src, got))
            if got == want:
                return t
            st[got] = t

    def _issue(self, recv=None):
        """Issue the queued payload sends (and ``recv`` = (tensor, src, tag)) as one batched p2p group; the receive is
        waited for (a stream wait on RCCL, host wait on gloo), the sends join the pending list."""
        sends, self.queued = self.queued, []
        if not sends and recv is None:
            return
        me = dist.get_rank() if dist.is_initialized() else 0
        ops = [("s", t, dst, tg, me < dst) for t, dst, tg in sends]
        if recv is not None:
            ops.append(("r", recv[0], recv[1], recv[2], recv[1] < me))
        batches = {}  # direction (to a higher rank?) -> ops, in order of first appearance (sends first)
        for op in ops:
            batches.setdefault(op[4], []).append(op)
        from ..distributed import collective_check as _cc
        rwork = None
        for up, bops in batches.items():
            pg = self.pg if up else self.pg_down
            if self.record:
                self.log.append(tuple((k, peer, tg) for k, _t, peer, tg, _u in bops))
            self.groups += 1
            if _cc.enabled() or len(bops) == 1:
                # one op, or the collective checker (debug mode): one by one, each under its own tag label (the
                # checker fingerprints every payload; P2POp takes only the unwrapped isend)
                works = []
                for k, t, peer, tg, _u in bops:
                    with self._label(tg):
                        works.append((dist.isend if k == "s" else dist.irecv)(t, peer, group=pg))
            else:
                # P2POp takes the c10d functions themselves (the checker / watchdog may have wrapped dist.isend)
                from torch.distributed import distributed_c10d as c10d
                works = dist.batch_isend_irecv([dist.P2POp(c10d.isend if k == "s" else c10d.irecv, t, peer,
                                                           group=pg) for k, t, peer, _tg, _u in bops])
            for (k, t, _p, _tg, _u), w in zip(bops, works):
                if k == "s":
                    self.pending.append((w, t))
                else:
                    rwork = w
        if rwork is not None:
            rwork.wait()

    def flush(self):
        """Issue the queued sends now (a schedule job that receives nothing calls this before its compute)."""
        self._issue(None)

    def join(self):
        self._issue(None)
        for w, _ in self.pending:
            w.wait()
        self.pending = []
