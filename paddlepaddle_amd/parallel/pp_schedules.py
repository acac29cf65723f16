"""Pipeline schedules as per-stage job lists (reference: distributed/passes/pipeline_scheduler_pass/
pipeline_1f1b.py, pipeline_fthenb.py, pipeline_zero_bubble.py:61 ZBH1 — job lists of forward / backward /
backward_b / backward_w per stage).

A job is (kind, micro_batch) with kind "F" (forward), "B" (backward: input gradients, and weight gradients
too unless the schedule splits them) or "W" (the deferred weight-gradient GEMMs of a micro-batch; see
ops/linear.py defer_weight_grads). Both pipeline engines (parallel/pipeline.py dygraph PipelineParallel and
distributed/auto_parallel/static_engine.py) execute these lists.

ZBH1 (zero bubble, "handcrafted 1"): 1F1B order for F and B, with W split off. During the steady phase a
stage keeps at most ``warm = stages - stage - 1`` W jobs pending (the same activation bound as 1F1B: each
pending W holds one micro-batch's linear inputs and output gradients); in the cool-down every B is followed
by one W, and the remaining W jobs run after the last B. The cool-down bubbles of 1F1B — a stage waiting
for the next output gradient from downstream — are filled with weight-gradient GEMMs, and the gradient
reaches the previous stage one W earlier per hop than with a fused backward.
"""
from __future__ import annotations

__all__ = ["schedule", "fthenb", "one_f_one_b", "eager_1f1b", "zbh1", "vpp", "zbvpp", "vpp_chunk", "vpp_mb",
           "SCHEDULES"]


def fthenb(n_stages, stage, n_mb):
    return [("F", i) for i in range(n_mb)] + [("B", i) for i in range(n_mb)]


def one_f_one_b(n_stages, stage, n_mb):
    warm = min(n_stages - stage - 1, n_mb)
    out = [("F", i) for i in range(warm)]
    fi, bi = warm, 0
    while fi < n_mb:
        out += [("F", fi), ("B", bi)]
        fi += 1
        bi += 1
    out += [("B", i) for i in range(bi, n_mb)]
    return out


def eager_1f1b(n_stages, stage, n_mb):
    """1F1B with 2 * (stages - stage) - 1 warm-up forwards (reference pipeline_eager_1f1b.py): one more
    activation in flight per hop than 1F1B, so a stage's next forward input is already on its way while it runs
    a backward (send / receive overlap); steady phase B then F."""
    warm = min(2 * (n_stages - stage) - 1, n_mb)
    out = [("F", i) for i in range(warm)]
    fi, bi = warm, 0
    while fi < n_mb:
        out += [("B", bi), ("F", fi)]
        fi += 1
        bi += 1
    out += [("B", i) for i in range(bi, n_mb)]
    return out


def zbh1(n_stages, stage, n_mb):
    warm = min(n_stages - stage - 1, n_mb)
    out = [("F", i) for i in range(warm)]
    pending = []
    fi, bi = warm, 0
    while fi < n_mb:
        out += [("F", fi), ("B", bi)]
        pending.append(bi)
        fi += 1
        bi += 1
        if len(pending) > warm:
            out.append(("W", pending.pop(0)))
    while bi < n_mb:
        out.append(("B", bi))
        pending.append(bi)
        bi += 1
        out.append(("W", pending.pop(0)))
    out += [("W", i) for i in pending]
    return out


def vpp(n_stages, stage, n_mb, n_chunks):
    """Interleaved 1F1B over ``n_chunks`` model chunks per stage (reference pipeline_vpp.py): jobs ("F", k) /
    ("B", k) over virtual micro-steps k in [0, n_mb * n_chunks); vpp_chunk / vpp_mb map k to (chunk, micro-batch):
    groups of ``n_stages`` micro-batches walk the chunks in order (forward) or reverse order (backward)."""
    if n_mb % n_stages:
        raise ValueError(f"accumulate_steps ({n_mb}) must be a multiple of the pipeline degree ({n_stages})")
    total = n_mb * n_chunks
    warm = min((n_stages - stage - 1) * 2 + (n_chunks - 1) * n_stages, total)
    out = [("F", k) for k in range(warm)]
    for i in range(total - warm):
        out += [("F", warm + i), ("B", i)]
    out += [("B", k) for k in range(total - warm, total)]
    return out


def zbvpp(n_stages, stage, n_mb, n_chunks):
    """Zero-bubble interleaved schedule (reference pipeline_scheduler_pass/pipeline_zero_bubble.py ZBVPP): the VPP
    order of forward / input-gradient jobs over virtual micro-steps, with each step's weight gradients split off
    as ("W", k) jobs the way zbh1 places them — during the steady phase at most ``stages - stage - 1`` W jobs stay
    pending (the 1F1B activation bound), each cool-down backward is followed by one W (the W GEMMs fill the
    bubbles while the stage waits for the next gradient from downstream), the rest run after the last backward."""
    base = vpp(n_stages, stage, n_mb, n_chunks)
    total = n_mb * n_chunks
    warm = min((n_stages - stage - 1) * 2 + (n_chunks - 1) * n_stages, total)
    bound = n_stages - stage - 1
    out, pending = [], []
    for kind, k in base:
        out.append((kind, k))
        if kind != "B":
            continue
        pending.append(k)
        if k >= total - warm or len(pending) > bound:  # cool-down backward, or over the steady-phase bound
            out.append(("W", pending.pop(0)))
    out += [("W", k) for k in pending]
    return out


def vpp_chunk(k, n_stages, n_chunks, forward=True):
    v = (k // n_stages) % n_chunks
    return v if forward else n_chunks - 1 - v


def vpp_mb(k, n_stages, n_chunks):
    return (k // (n_stages * n_chunks)) * n_stages + k % n_stages


SCHEDULES = {"FTHENB": fthenb, "1F1B": one_f_one_b, "EAGER1F1B": eager_1f1b, "ZBH1": zbh1}


def schedule(mode, n_stages, stage, n_mb):
    fn = SCHEDULES.get(str(mode).upper())
    if fn is None:
        raise ValueError(f"unknown pipeline schedule {mode!r}; one of {sorted(SCHEDULES)}")
    return fn(n_stages, stage, n_mb)


def check(jobs, n_mb, split_w):
    """Validity of one stage's job list: every micro-batch forwarded once, backward after its forward, W after
    its B (and present exactly when the schedule splits weight gradients)."""
    seen = {}
    for pos, (k, mb) in enumerate(jobs):
        if (k, mb) in seen:
            raise AssertionError(f"duplicate job {(k, mb)}")
        seen[(k, mb)] = pos
    for mb in range(n_mb):
        assert seen[("F", mb)] < seen[("B", mb)], mb
        if split_w:
            assert seen[("B", mb)] < seen[("W", mb)], mb
        else:
            assert ("W", mb) not in seen
    return True
