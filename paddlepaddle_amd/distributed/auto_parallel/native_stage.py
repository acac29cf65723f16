"""A static auto-parallel engine's stage program on the native training executor (csrc/interpreter/train_interp.cpp).

Reference: auto_parallel/static/engine.py runs each rank's partitioned program on the standalone executor
(new_executor/pir_interpreter.cc). Here a virtual stage's local op list (static_engine._LNode items: the traced
global program after placement propagation and partition, collectives explicit) is lowered once, after its first
micro-batch ran in Python, into one TrainProgram whose ``forward`` runs the micro-batch in C++:

  * hot ops of this framework (fused_linear, linear_nt, layer_norm / rms_norm, flash attention, softmax-CE, NHWC
    conv / BN) become native instructions — C++ autograd nodes on the hand-written kernels;
  * the other ops of this framework (qkv_rope_attention, swiglu, rms_norm_residual, ...), every collective with its
    autograd conjugate (allreduce / allgather / slice / reduce_scatter / copy_to_parallel / vocab-parallel CE and
    embedding) and linears with a tensor-parallel dX hook are Python-call instructions (their kernels and
    collectives unchanged);
  * torch-level ops become boxed ATen dispatcher calls captured on meta tensors of the shapes the first
    micro-batch produced.

Recompute segments are one Python-call instruction each (the engine's checkpointed run of the segment). The
backward stays the caller's (torch autograd over what the instructions recorded); p2p sends / receives and the
schedule stay in the engine. Under the zero-bubble schedules the linears stay Python calls (their deferred
weight-gradient GEMMs live in ops/linear.py).
"""
from __future__ import annotations

import torch

from ...static import native_train as NT

__all__ = ["compile_stage", "NativeStage"]


class _Node:
    """The attribute view of an engine _LNode that the lowering expects."""
    __slots__ = ("func", "args", "kwargs", "outs", "name", "kind")

    def __init__(self, nd):
        self.func, self.args, self.kwargs, self.outs, self.name, self.kind = nd.fn, nd.args, nd.kwargs, nd.outs, \
            nd.name, "op"


class _StageProg:
    """What _Lowering reads of a program: the meta tensor of every slot."""

    def __init__(self, metas):
        self._metas = metas


def _has_engine_tmpl(t):
    from .static_engine import _HookT
    if isinstance(t, _HookT):
        return True
    if isinstance(t, tuple) and len(t) == 3 and t[0] == "G":
        return True
    if isinstance(t, (list, tuple)):
        return any(_has_engine_tmpl(v) for v in t)
    if isinstance(t, dict):
        return any(_has_engine_tmpl(v) for v in t.values())
    return False


class NativeStage:
    def __init__(self, tp, feed_slots, fetch, n_native, n_py, low):
        self.tp = tp
        self.feed_slots = feed_slots   # slots fed on every call (parameters, feeds, received activations)
        self.fetch = fetch
        self.num_native, self.num_py = n_native, n_py
        self.num_instructions = tp.num_instructions
        self._low = low  # keeps bound constants alive
        self.runs = 0

    def forward(self, env):
        """env: slot -> tensor for the feed slots; returns {fetch slot: tensor with autograd history}."""
        outs = self.tp.forward([(s, env[s]) for s in self.feed_slots if s in env])
        self.runs += 1
        return dict(zip(self.fetch, outs))


def compile_stage(eng, s, env, fetch, python_linears=False):
    """Lower virtual stage ``s`` of engine ``eng`` using the values its first micro-batch left in ``env`` (their
    shapes / dtypes); ``fetch``: the slots the engine reads after the stage (sends, loss); ``python_linears``: the
    linears stay Python-call instructions (the zero-bubble schedules defer their weight-gradient GEMMs through
    ops/linear.py). Returns (NativeStage, None) or (None, reason)."""
    m = NT._module()
    if m is None:
        return None, "_C_train not built"
    from .static_engine import _Seg, _flat_tensor_refs
    items = eng.stage_items[s]
    with torch._C.DisableTorchFunction():
        top = max([k for k in env] + [0]) + 1
        metas = [None] * top
        for k, v in env.items():
            if isinstance(v, torch.Tensor):
                # the exact strides (views such as the q / k / v slices of a fused projection are not dense): an op
                # replayed on the meta decides view vs copy the way it will at run time
                metas[k] = torch.empty_strided(v.size(), v.stride(), dtype=v.dtype,
                                               device="meta").requires_grad_(v.requires_grad)
    dev = next((v.device for v in env.values() if isinstance(v, torch.Tensor)), torch.device("cpu"))
    gpu = dev.type == "cuda"  # the native kinds launch HIP kernels: on CPU every op of ours is a Python call
    low = NT._Lowering(_StageProg(metas), dev, gpu)
    produced = set()
    n_native = n_py = 0
    try:
        with NT._NoTrace():
            for nd in items:
                if isinstance(nd, _Seg):  # a recompute segment: one Python call of the engine's checkpointed run
                    def seg_call(*ts, seg=nd):
                        e = dict(zip(seg.inputs, ts))
                        eng._run_segment(seg, e)
                        return tuple(e[o] for o in seg.outputs)
                    low.instrs.append(("py", seg_call, list(nd.inputs), list(nd.outputs), "recompute_segment"))
                    produced.update(nd.outputs)
                    n_py += 1
                    continue
                node = _Node(nd)
                outs = [r.i for r in _flat_tensor_refs(nd.outs, [])] if nd.outs is not None else []
                if nd.outs is None:
                    return None, f"in-place op {nd.name}"
                ours = nd.name.startswith("o:")
                lin = python_linears and nd.name.rsplit(":", 1)[-1] in ("fused_linear", "linear_nt")
                if gpu and not lin and not _has_engine_tmpl((nd.args, nd.kwargs)) and ours and low.lower_native(node):
                    n_native += 1
                elif ours or _has_engine_tmpl((nd.args, nd.kwargs)) or not nd.name.startswith(("f:", "m:", "p:")):
                    fn, sa, a, sk, k, _oi, _o = eng._compile_node(nd)
                    refs = [r.i for r in _flat_tensor_refs((nd.args, nd.kwargs), [])]

                    def call(*ts, fn=fn, sa=sa, a=a, sk=sk, k=k, refs=refs):
                        e = dict(zip(refs, ts))
                        return fn(*(a if sa else a(e)), **(k if sk else k(e)))
                    low.instrs.append(("py", call, refs, outs, nd.name))
                    n_py += 1
                else:
                    low.lower_generic(node)
                produced.update(outs)
    except NT.Unsupported as e:
        return None, str(e)
    except Exception as e:  # noqa: BLE001 - an op the meta replay cannot run
        return None, f"lowering failed: {type(e).__name__}: {e}"
    tp = m.TrainProgram(low.n, str(low.dev))
    try:
        for ins in low.instrs:
            if ins[0] == "aten":
                tp.add_aten(f"{ins[1]}", ins[2], [tuple(a) for a in ins[3]], ins[4])
            elif ins[0] == "py":
                tp.add_py(ins[1], ins[2], ins[3], ins[4])
            else:
                tp.add_native(ins[1], ins[2], ins[3], ins[4], ins[5])
    except Exception as e:  # noqa: BLE001
        return None, f"instruction build failed: {type(e).__name__}: {e}"
    for slot, t in low.binds.items():
        tp.bind(slot, t)
    missing = [f for f in fetch if f not in produced and f not in env]
    if missing:
        return None, f"fetch slots {missing} not produced by the stage"
    tp.finalize(list(fetch))
    feeds = sorted(k for k in env if k not in produced)
    return NativeStage(tp, feeds, list(fetch), n_native, n_py, low), None
