"""Pipeline communication programs and a rendezvous replay that proves a schedule cannot deadlock on RCCL.

RCCL / NCCL point-to-point operations are rendezvous: a send completes only while the matching receive is posted
on the peer, messages between a pair match in issue order, and the ops of one rank pair run on one stream in
issue order. gloo buffers sends, so a pattern that hangs on RCCL can pass every CPU test. This module derives, for
a pipeline schedule (parallel/pp_schedules.py job lists), the exact sequence of p2p groups each stage issues —
the rule parallel/p2p.py and both pipeline engines follow:

* a job's payload receive is issued together with the payload sends still queued from the previous job, as one
  batched group (batch_isend_irecv, reference pp_utils/p2p_communication.py:286, :573);
* a job that receives nothing (first stage's forwards, last stage's backwards, W jobs) flushes the queued sends
  before its compute; the end of the run flushes the rest;
* headers (tensor meta on the gloo host twin) go out when a send is queued; before its host blocks on reading one,
  a receiver issues its queued sends on their own; a receiver whose host must read one
  (the first message of each class per run in ordered mode, every message in the tagged mode of the interleaved
  schedules, which also stashes messages that arrive ahead of the one it needs) blocks its host until the sender
  has queued that send —

* payloads to a higher rank travel on one communicator, to a lower rank on another, so a stream never carries a
  rank pair's sends and receives; a batched group is issued as one batch per direction —

and ``simulate`` replays those programs under rendezvous semantics: per rank, the host issues groups in program
order (blocked only by header reads); on the device a group starts once every receive of the rank's earlier
groups has completed (the compute stream orders every op after the data it consumes) and once it is at the head
of every pair stream it uses; a posted send and the posted receive of the same message complete together. A
program set that ends with ops left and no move possible deadlocks. ``batched=False`` builds the previous,
ungrouped protocol (each send its own isend at the end of the job) for comparison.
"""
from __future__ import annotations

import collections

from .pp_schedules import schedule, vpp, vpp_chunk, vpp_mb, zbvpp

__all__ = ["programs", "simulate", "Deadlock"]


class Deadlock(RuntimeError):
    pass


def _chain_msgs(mode, S, M):
    """(jobs per stage, per-job (recv msgs, send msgs)) of a non-interleaved pipeline of S stages."""
    jobs = [schedule(mode, S, s, M) for s in range(S)]
    comm = []
    for s in range(S):
        cs = []
        for kind, mb in jobs[s]:
            if kind == "F":
                rcv = [(s - 1, s, ("F", 0, mb))] if s > 0 else []
                snd = [(s, s + 1, ("F", 0, mb))] if s < S - 1 else []
            elif kind == "B":
                rcv = [(s + 1, s, ("B", 0, mb))] if s < S - 1 else []
                snd = [(s, s - 1, ("B", 0, mb))] if s > 0 else []
            else:  # W: no communication
                rcv, snd = [], []
            cs.append((rcv, snd))
        comm.append(cs)
    return comm


def _vpp_msgs(S, M, V, zb=False):
    """Interleaved 1F1B over V chunks per stage (ring), in the message keys of parallel/pipeline.py; zb: the ZBVPP
    order (W jobs communicate nothing)."""
    comm = []
    for s in range(S):
        cs = []
        for kind, k in (zbvpp if zb else vpp)(S, s, M, V):
            if kind == "W":
                cs.append(([], []))
                continue
            if kind == "F":
                v, mb = vpp_chunk(k, S, V, True), vpp_mb(k, S, V)
                first, last = s == 0 and v == 0, s == S - 1 and v == V - 1
                rcv = [] if first else [((s - 1) % S, s, ("F", v if s else v - 1, mb))]
                snd = [] if last else [(s, (s + 1) % S, ("F", v, mb))]
            else:
                v, mb = vpp_chunk(k, S, V, False), vpp_mb(k, S, V)
                first, last = s == 0 and v == 0, s == S - 1 and v == V - 1
                rcv = [] if last else [((s + 1) % S, s, ("B", v + 1 if s == S - 1 else v, mb))]
                snd = [] if first else [(s, (s - 1) % S, ("B", v, mb))]
            cs.append((rcv, snd))
        comm.append(cs)
    return comm


def programs(mode, S, M, V=1, batched=True, ordered=None, split_directions=True):
    """Per-stage p2p programs: programs[s] = list of groups; a group is a list of ops
    ("s" | "r", src, dst, msg, header_needed). ``msg`` = (src, dst, key) identifies a message. split_directions: a
    batched group is issued as one batch per direction (to a higher / lower rank: two communicators), sends'
    directions first — what parallel/p2p.py does."""
    mode = str(mode).upper()
    comm = _vpp_msgs(S, M, V, mode == "ZBVPP") if mode in ("VPP", "ZBVPP") else _chain_msgs(mode, S, M)
    ordered = (mode not in ("VPP", "ZBVPP")) if ordered is None else ordered
    # production order of every directed channel (the order the sender queues its messages)
    prod = collections.defaultdict(list)
    for s in range(S):
        for _rcv, snd in comm[s]:
            for src, dst, key in snd:
                prod[(src, dst)].append(key)
    progs = []
    for s in range(S):
        groups, queued = [], []
        seen_class = set()
        consumed = collections.defaultdict(set)   # tagged mode: messages already received (stash)
        pos = collections.defaultdict(int)        # tagged mode: next production index read per channel
        for rcv, snd in comm[s]:
            ops = []
            for src, dst, key in rcv:
                if ordered:
                    cls = (src, key[0])
                    hdr = cls not in seen_class
                    seen_class.add(cls)
                    ops.append(("r", src, dst, (src, dst, key), hdr))
                else:
                    if key in consumed[(src, dst)]:
                        consumed[(src, dst)].discard(key)
                        continue
                    seq = prod[(src, dst)]
                    while True:  # read headers in production order until the wanted message, stashing the rest
                        got = seq[pos[(src, dst)]]
                        pos[(src, dst)] += 1
                        ops.append(("r", src, dst, (src, dst, got), True))
                        if got == key:
                            break
                        consumed[(src, dst)].add(got)
            if batched:
                if ops:
                    if ops[0][4] and queued:  # the host blocks on a header read: the queued sends go out first
                        groups.append(queued)
                        queued = []
                    groups.append(queued + [ops[0]])
                    groups.extend([o] for o in ops[1:])
                    queued = []
                elif queued and not rcv:  # a job without a receive flushes; one served from the stash keeps them
                    groups.append(queued)
                    queued = []
                queued = queued + [("s", src, dst, (src, dst, key), False) for src, dst, key in snd]
            else:
                groups.extend([o] for o in ops)
                groups.extend([("s", src, dst, (src, dst, key), False)] for src, dst, key in snd)
        if queued:
            groups.append(queued)
        if split_directions:
            split = []
            for g in groups:
                by = {}
                for op in g:
                    by.setdefault(op[3][0] < op[3][1], []).append(op)
                split.extend(by.values())
            groups = split
        progs.append(groups)
    return progs


def _stream(op, per_direction):
    peer = op[2] if op[0] == "s" else op[1]
    return (peer, op[3][0] < op[3][1]) if per_direction else peer


def simulate(progs, per_direction=True, host_waits=False, max_rounds=10 ** 7):
    """Replay the programs under rendezvous semantics; returns the number of matched messages, raises Deadlock.
    per_direction: one stream per (rank pair, direction) — the two payload communicators of parallel/p2p.py;
    False: one stream per rank pair (a single communicator). host_waits: a receive also blocks the host until
    its data arrived (gloo; on RCCL the wait is a stream wait)."""
    R = len(progs)
    issued = [0] * R                       # host: groups issued per rank
    queue_pt = {}                          # message -> (sender, index of the group that carries it)
    for r, gs in enumerate(progs):
        for gi, g in enumerate(gs):
            for op in g:
                if op[0] == "s":
                    queue_pt[op[3]] = (r, gi)
    streams = collections.defaultdict(collections.deque)  # (rank, peer) -> deque of (group index, op index)
    done = [[[False] * len(g) for g in gs] for gs in progs]
    started = [[False] * len(gs) for gs in progs]
    recv_done_upto = [0] * R               # every receive of groups < this index has completed
    posted = {}                            # (msg, kind) -> (rank, group, op)
    total = sum(len(g) for gs in progs for g in gs)
    completed = 0

    def header_ready(r, g):
        for op in progs[r][g]:
            if op[0] == "r" and op[4]:
                src, gi = queue_pt[op[3]]
                # the sender queues the send (and its header) after issuing group gi - 1
                if issued[src] < gi:
                    return False
        return True

    for _ in range(max_rounds):
        moved = False
        for r in range(R):  # host issue
            while issued[r] < len(progs[r]) and header_ready(r, issued[r]) and (
                    not host_waits or issued[r] == 0 or all(
                        done[r][issued[r] - 1][oi] or op[0] == "s" for oi, op in enumerate(progs[r][issued[r] - 1]))):
                gi = issued[r]
                for oi, op in enumerate(progs[r][gi]):
                    streams[(r, _stream(op, per_direction))].append((gi, oi))
                issued[r] += 1
                moved = True
        for r in range(R):  # device: start groups
            while recv_done_upto[r] < issued[r] and all(
                    done[r][recv_done_upto[r]][oi] or progs[r][recv_done_upto[r]][oi][0] == "s"
                    for oi in range(len(progs[r][recv_done_upto[r]]))):
                recv_done_upto[r] += 1
            for gi in range(issued[r]):
                if started[r][gi] or gi > recv_done_upto[r]:
                    continue
                # the group's ops must lead every pair stream they are on (a group may hold several ops of one
                # stream, e.g. a send to and a receive from the same neighbour)
                need = collections.Counter()
                for op in progs[r][gi]:
                    need[_stream(op, per_direction)] += 1
                heads = True
                for peer, n in need.items():
                    dq = streams[(r, peer)]
                    if len(dq) < n or any(dq[i][0] != gi for i in range(n)):
                        heads = False
                        break
                if not heads:
                    continue
                started[r][gi] = True
                moved = True
                for oi, op in enumerate(progs[r][gi]):
                    posted[(op[3], op[0])] = (r, gi, oi)
        for (msg, kind), (r, gi, oi) in list(posted.items()):  # match
            if kind != "s" or (msg, "s") not in posted:
                continue
            other = posted.get((msg, "r"))
            if other is None:
                continue
            for (rr, gg, oo) in ((r, gi, oi), other):
                done[rr][gg][oo] = True
                streams[(rr, _stream(progs[rr][gg][oo], per_direction))].remove((gg, oo))
            del posted[(msg, "s")]
            del posted[(msg, "r")]
            completed += 2
            moved = True
        if completed == total:
            return total // 2
        if not moved:
            left = [(r, gi, progs[r][gi]) for r in range(R) for gi in range(len(progs[r]))
                    if not all(done[r][gi])][:6]
            raise Deadlock(f"no progress with {total - completed} of {total} ops pending; host issued "
                           f"{issued}; first pending groups: {left}")
    raise Deadlock("simulation did not finish")
