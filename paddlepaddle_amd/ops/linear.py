"""Linear layers with fused epilogues.

Reference: paddle/phi/kernels/fusion/gpu/fused_gemm_epilogue_kernel.cu (+_grad),
python/paddle/incubate/nn/functional/fused_matmul_bias.py.
paddle's Linear weight is [in_features, out_features]: y = x @ W + b.

MI355X path (one autograd node per linear):
  forward : y = x W (+b) on either the hand-written MFMA GEMM (csrc/kernels/gemm.hip: bias and
            tanh-GELU fused into the epilogue, pre-activation stored for the backward) or hipBLASLt
            (addmm, then a HIP bias+GELU pass) — per shape, whichever measured faster on first use
            (ops/gemm.py choose()).
  backward: dX = dY Wᵀ and dW = Xᵀ dY on the same per-shape choice; the hand-written kernel reads
            the transposed operands in place (MN-major LDS images + ds_read_b64_tr_b16) and accumulates
            dW straight into the sharding engine's grad buffer. The bias gradient is a HIP column
            reduction (csrc/kernels/linear_epi.hip) and, for GELU, one fused pass produces
            dH = dY·gelu'(h + b) together with db.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _loader as L
from . import dropout as _dropout
from . import gemm as G
from .activation import bias_gelu, gelu
from ..framework.trace_hook import static_op


def colsum(x2d, acc=None):
    """Column sums of a [rows, cols] tensor (bias gradient); added in place into ``acc`` when given. A gradient
    whose producer (a dropout backward) already wrote its column partials only has them folded."""
    rows, cols = x2d.shape
    pre = _dropout.take_colsum(x2d) if x2d.is_cuda else None
    if pre is not None:
        out = acc if acc is not None else torch.empty(cols, dtype=x2d.dtype, device=x2d.device)
        L.call("pa_fold_partials", L.ptr(pre[0]), L.ptr(out), cols, pre[1], L.dcode(x2d) | ((acc is not None) << 8),
               L.stream_ptr())
        return out
    if L.hip_enabled_for(x2d) and x2d.dtype in L._DT and cols % 8 == 0 and x2d.is_contiguous():
        out = acc if acc is not None else torch.empty(cols, dtype=x2d.dtype, device=x2d.device)
        ws = torch.empty(256 * cols, dtype=torch.float32, device=x2d.device)
        L.call("pa_colsum", L.ptr(x2d), L.ptr(out), L.ptr(ws), rows, cols,
               L.dcode(x2d) | ((acc is not None) << 8), L.stream_ptr())
        return out
    s = x2d.float().sum(0).to(x2d.dtype)
    return s if acc is None else acc.add_(s)


def _vector_main_grad(p, dtype):
    """(buffer, ready handler) when ``p``'s gradient accumulates in place (main-grad fusion for biases / norm
    parameters: the finalize kernels add into the buffer), else None."""
    ent = _main_grad_of(p) if p is not None else None
    if ent is None or ent[1].dtype != dtype or not ent[1].is_contiguous():
        return None
    return ent[1], ent[2]


# ---------------------------------------------------------------------------------------------
# Forward-weight layout cache. hipBLASLt on gfx950 runs y = x @ W 10-30% faster in the "TN" form
# (W stored [out, in], read transposed) than in the "NN" form for the GPT/LLaMA linear shapes
# (tools/bench_gemm.py: fc2 4096x20480x5120 0.86 ms -> 0.66 ms), while the data-gradient
# dX = dY @ W^T is already fastest with paddle's [in, out] storage. So parameters keep paddle's
# layout and the forward reads a per-step [out, in] copy: made once per weight per optimizer step
# (weights only change in step(); gradient-accumulation micro-batches reuse it), dropped when any
# optimizer steps (bump_weight_epoch), bounded by FLAGS_linear_wt_cache_mb.
# Measured on the full GPT-3 13B step (profiles/gpt13b_sharding3_1gpu.md vs a run with the cache on):
# the isolated-GEMM gain does not survive sustained load (GEMM time 6.16 s vs 6.21 s per 3 steps, plus
# ~54 ms/step of transposes), so it is off by default and kept for shapes where it does pay.
_WT = {}
_WT_BYTES = [0]


def bump_weight_epoch():
    _WT.clear()
    _WT_BYTES[0] = 0


def _fwd_weight(w):
    if w.dim() != 2 or not w.is_cuda:
        return None
    ent = _WT.get(id(w))
    if ent is not None and ent[0]() is w and ent[1] == w._version and ent[2] == w.data_ptr():
        return ent[3]
    nbytes = w.numel() * w.element_size()
    if _WT_BYTES[0] + nbytes > L.flag("FLAGS_linear_wt_cache_mb", 0) * (1 << 20):
        return None
    import weakref
    wt = w.t().contiguous()
    if ent is not None:
        _WT_BYTES[0] -= ent[3].numel() * ent[3].element_size()
    _WT[id(w)] = (weakref.ref(w), w._version, w.data_ptr(), wt)
    _WT_BYTES[0] += nbytes
    return wt


def _blas_fwd(x2, w, b=None):
    wt = _fwd_weight(w)
    wv = wt.t() if wt is not None else w
    return torch.addmm(b, x2, wv) if b is not None else torch.mm(x2, wv)


def _fwd_mm_res(x2, w, b, r2):
    """x2 @ w (+ b) + r2: the residual add in the GEMM (hand-written epilogue, or hipBLASLt's beta = 1 C input),
    timed per shape like every other forward GEMM."""
    if G.res_supported(x2, w, r2):
        key = ("fwd_res", x2.shape[0], w.shape[1], x2.shape[1], b is not None)

        def blas():
            y = torch.addmm(r2, x2, w)
            return y.add_(b) if b is not None else y
        if G.choose(key, {"blas": blas, "hip": lambda: G.gemm_res(x2, w, r2, bias=b)}) == "hip":
            return G.gemm_res(x2, w, r2, bias=b)
        return blas()
    return _fwd_mm(x2, w, b).add_(r2)


def _fwd_mm(x2, w, b=None):
    if x2.shape[0] <= 64 and G.small_m_supported(x2, w):
        M, K, N = x2.shape[0], x2.shape[1], w.shape[1]
        key = ("fwd_small_m", M, N, K, b is not None)
        cands = {"blas": lambda: _blas_fwd(x2, w, b)}
        for d, st in G.small_m_variants(M, N, K):
            cands[f"hip_s{d}_st{st}"] = (lambda d=d, st=st: G.gemm_small_m(x2, w, b, splits=d, stages=st))
        ch = G.choose(key, cands, cold=True)
        if ch.startswith("hip"):
            if ch == "hip":  # FLAGS_gemm_backend=hip: default split heuristic
                return G.gemm_small_m(x2, w, b)
            d, st = (int(v[1:]) for v in ch[4:].replace("st", "t").split("_"))
            return G.gemm_small_m(x2, w, b, splits=d, stages=st)
        return _blas_fwd(x2, w, b)
    if G.supported(x2, w):
        key = ("fwd", x2.shape[0], w.shape[1], x2.shape[1], b is not None)
        ch = G.choose(key, {"blas": lambda: _blas_fwd(x2, w, b), "hip": lambda: G.gemm(x2, w, bias=b)})
        if ch == "hip":
            return G.gemm(x2, w, bias=b)
    return _blas_fwd(x2, w, b)


def _fwd_bias_gelu(x2, w, b):
    """(y, pre, bias_for_bwd): y = gelu(x2 @ w + b); pre / bias_for_bwd feed pa_bias_gelu_bwd."""
    if G.supported(x2, w):
        M, N = x2.shape[0], w.shape[1]

        def hip():
            pre = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
            return G.gemm(x2, w, bias=b, gelu=True, aux=pre), pre

        def blas():
            h = _blas_fwd(x2, w)
            return bias_gelu(h, b), h
        ch = G.choose(("fwd_gelu", M, N, x2.shape[1]), {"blas": blas, "hip": hip})
        if ch == "hip":
            y, pre = hip()
            return y, pre, torch.zeros_like(b)
    h = _blas_fwd(x2, w)
    return bias_gelu(h, b), h, b


# ---------------------------------------------------------------------------------------------
# Gradient-accumulation fusion. An engine that owns flat gradient buffers (parallel/sharding.py) can
# register a weight together with the slice of its buffer that holds that weight's gradient; the
# weight-gradient GEMM then accumulates straight into it (hipBLASLt beta = 1) instead of producing a
# fresh dW that autograd adds into .grad in a second full-size pass (~4 % of the 13B step). Because
# autograd then sees no gradient for the weight, the engine also passes the grad-ready handler its
# post-accumulate hook would have run; it is invoked with the weight after the in-place GEMM.
import weakref  # noqa: E402

_MAIN_GRAD = {}  # id(weight) -> (weakref to weight, grad buffer view, ready handler)


def register_main_grad(weight, buffer, on_ready):
    """Accumulate ``weight``'s gradient in place into ``buffer`` (same shape/dtype) and call
    ``on_ready(weight)`` afterwards. Used by GroupShardedEngine for the flat grad buffers."""
    if buffer.shape != weight.shape or buffer.dtype != weight.dtype:
        raise ValueError("main-grad buffer must match the weight's shape and dtype")
    key = id(weight)

    def _drop(ref):  # the weight died: release its buffer view (engines re-create weights, e.g. ZeRO-3 gathers)
        ent = _MAIN_GRAD.get(key)
        if ent is not None and ent[0] is ref:
            del _MAIN_GRAD[key]
    _MAIN_GRAD[key] = (weakref.ref(weight, _drop), buffer, on_ready)


_FUSE_TYPES = ("Linear", "ColumnParallelLinear", "RowParallelLinear", "LlamaRMSNorm", "RMSNorm", "LayerNorm",
               "FusedLinear")


def fuse_grad_accumulation(layer, params=None):
    """Fused gradient accumulation (reference: fused_linear_param_grad_add_kernel.cu:146 / PaddleNLP main_grad):
    the .grad buffer of every linear / norm parameter of ``layer`` is registered as its main-grad, so each
    backward's weight-gradient GEMM adds into it in its epilogue (and the norm backward kernels add their column
    sums) instead of autograd allocating a fresh dW and adding it into .grad with a separate pass. Parameters used
    by more than one layer (tied weights) or owned by other layer types keep autograd accumulation. Call once per
    step before the backwards (cheap: re-registers only buffers an optimizer replaced); pass the returned list back
    as ``params``. The optimizer must clear gradients with set_to_zero=True (the default). Disabled by
    FLAGS_fused_grad_accumulation=0."""
    from ..framework.flags import flag
    if not flag("FLAGS_fused_grad_accumulation", True):
        return params or []
    if params is None:
        owners = {}
        for sub in layer.sublayers(include_self=True):
            for name, p in sub.named_parameters(include_sublayers=False):
                owners.setdefault(id(p), []).append((type(sub).__name__, name, p))
        params = []
        for lst in owners.values():
            tname, name, p = lst[0]
            if (len(lst) == 1 and tname in _FUSE_TYPES and name in ("weight", "bias") and not p.stop_gradient
                    and p._t.is_cuda and p._t.dim() in (1, 2) and p._t.dtype in (torch.bfloat16, torch.float16)):
                params.append(p)

    def ready(w):
        for h in (getattr(w, "_post_accumulate_grad_hooks", None) or {}).values():
            h(w)
    for p in params:
        t = p._t
        if t.grad is None:
            t.grad = torch.zeros_like(t)
        ent = _main_grad_of(t)
        if ent is None or ent[1].data_ptr() != t.grad.data_ptr():
            register_main_grad(t, t.grad, ready)
    return params


def unregister_main_grad(weight):
    _MAIN_GRAD.pop(id(weight), None)


_SAME = object()


def _main_grad_of(w):
    ent = _MAIN_GRAD.get(id(w))
    if ent is None or ent[0]() is not w:  # identity check: ids of dead tensors can be reused
        return None
    return ent


def _dgrad(dy2, w):
    wt = w.t()
    if G.supported(dy2, wt):
        key = ("dgrad", dy2.shape[0], wt.shape[1], dy2.shape[1])
        if G.choose(key, {"blas": lambda: torch.mm(dy2, wt), "hip": lambda: G.gemm(dy2, wt)}) == "hip":
            return G.gemm(dy2, wt)
    return torch.mm(dy2, wt)


def _wgrad(x2, dy2, acc=None):
    """x2^T @ dy2, accumulated in place into ``acc`` when given (main-grad fusion)."""
    xt = x2.t()
    if G.supported(xt, dy2):
        key = ("wgrad", xt.shape[0], dy2.shape[1], xt.shape[1], None if acc is None else acc.dtype)
        # few output tiles over a long K (weights of small layers, many tokens): the split-K ping-pong kernel
        sk = G.pp_splits(*key[1:4]) if -(-key[1] // 256) * -(-key[2] // 256) < 256 else 0
        sk = sk if G.gemm_pp_splitk_ok(xt, dy2, sk) and (acc is None or acc.is_contiguous()) else 0
        if acc is None:
            cands = {"blas": lambda: torch.mm(xt, dy2), "hip": lambda: G.gemm(xt, dy2)}
            if sk:
                cands["hip_sk"] = lambda: G.gemm_pp_splitk(xt, dy2, sk, dy2.dtype)
        else:
            scratch = []

            def _s():
                if not scratch:
                    scratch.append(torch.zeros_like(acc))
                return scratch[0]
            cands = {"blas": lambda: _s().addmm_(xt, dy2),
                     "hip": lambda: G.gemm(xt, dy2, out=_s(), accumulate=True)}
            if sk:
                cands["hip_sk"] = lambda: G.gemm_pp_splitk(xt, dy2, sk, out=_s(), accumulate=True)
        ch = G.choose(key, cands)
        if ch == "hip":
            if acc is None:
                return G.gemm(xt, dy2)
            G.gemm(xt, dy2, out=acc, accumulate=True)
            return acc
        if ch == "hip_sk":
            if acc is None:
                return G.gemm_pp_splitk(xt, dy2, sk, dy2.dtype)
            G.gemm_pp_splitk(xt, dy2, sk, out=acc, accumulate=True)
            return acc
    if acc is None:
        return torch.mm(xt, dy2)
    return acc.addmm_(xt, dy2)


# ---------------------------------------------------------------------------------------------
# Zero-bubble pipelining (parallel/pp_schedules.py ZBH1): the backward of a micro-batch is split into B
# (input gradients: on the critical path to the previous stage) and W (weight gradients: deferrable into
# the pipeline's cool-down bubbles). Inside ``defer_weight_grads(q)`` a linear's backward computes dX and
# the bias gradient and appends (weight, x, dY) to ``q`` instead of running the dW GEMM;
# ``apply_weight_grads(q)`` runs those GEMMs later (same main-grad / accumulate paths, then the weight's
# post-accumulate hooks). ``zero_bubble_forward()`` routes every linear through the deferrable autograd
# function for the forwards of such a schedule (off the HIP path a linear is otherwise a plain addmm).
import contextlib  # noqa: E402
import types  # noqa: E402

# Process-wide, not thread-local: the backward of cuda tensors may run on an autograd worker thread (torch's
# engine executes device nodes on a per-device thread), which must still see the queue of the B step.
_ZB = types.SimpleNamespace(queue=None, route=False)


@contextlib.contextmanager
def defer_weight_grads(queue):
    prev = getattr(_ZB, "queue", None)
    _ZB.queue = queue
    try:
        yield queue
    finally:
        _ZB.queue = prev


@contextlib.contextmanager
def zero_bubble_forward(enable=True):
    prev = getattr(_ZB, "route", False)
    _ZB.route = enable
    try:
        yield
    finally:
        _ZB.route = prev


def capture_forward_mode():
    """The op-routing state of the running forward (zero-bubble weight-gradient routing), for a recompute that
    re-runs this forward later inside backward: the recomputed ops must take the same path (same saved tensors)."""
    return {"zb": getattr(_ZB, "route", False)}


class forward_mode:
    """Re-enterable context applying a captured forward mode (a checkpoint may recompute a segment more than
    once, entering its recompute context each time)."""

    def __init__(self, mode):
        self.mode = mode
        self.prev = []

    def __enter__(self):
        self.prev.append(getattr(_ZB, "route", False))
        _ZB.route = self.mode["zb"]
        return self

    def __exit__(self, *exc):
        _ZB.route = self.prev.pop()
        return False


def apply_weight_grads(queue):
    """Run the deferred weight-gradient GEMMs of ``queue`` (in order) and clear it."""
    for w, x2, dy2 in queue:
        ent = _main_grad_of(w)
        if ent is not None and ent[1].dtype == dy2.dtype:
            _wgrad(x2, dy2, acc=ent[1])
            ent[2](w)
            continue
        if w.grad_fn is not None:
            # the linear read a derived weight (a cast / TP slice recorded in the program): dW flows back
            # through that chain to the parameter (B never entered it, so its saved tensors are intact)
            torch.autograd.backward(w, _wgrad(x2, dy2))
            continue
        if w.grad is None:
            w.grad = _wgrad(x2, dy2).to(w.dtype)
        elif w.grad.dtype == dy2.dtype and w.grad.is_contiguous():
            _wgrad(x2, dy2, acc=w.grad)
        else:
            w.grad.add_(_wgrad(x2, dy2))
        for h in (getattr(w, "_post_accumulate_grad_hooks", None) or {}).values():
            h(w)
    queue.clear()


# ---------------------------------------------------------------------------------------------
# Weight-gradient pairing across gradient-accumulation micro-batches. Every micro-batch of an accumulation window
# accumulates dW = x^T dY into the same main-grad buffer (K = the micro-batch's tokens); each such GEMM re-reads
# and re-writes the whole buffer and pays a round of tile prologues / epilogues. On MI355X the 288 GB of HBM hold
# one micro-batch's weight-gradient operands (x, dY of every linear: ~26 GB for GPT-3 13B at 4096 tokens), so
# inside ``pair_weight_grads("defer")`` a linear's main-grad dW GEMM is queued instead of run (its grad-ready
# hook waits too), and inside ``pair_weight_grads("merge")`` the next micro-batch's dW GEMM of the same weight
# runs as ONE two-segment product over K = 2T ([x_a | x_b]^T [dY_a ; dY_b], ops.gemm.gemm_seg: no concatenated
# copy), accumulated once. Leaving a "merge" region runs every job still queued on its own; a weight met twice in
# one "defer" region (tied weights) is paired right away. Reference: none (gradient accumulation in the
# reference accumulates per micro-batch, fleet/meta_parallel/sharding); an MI355X-memory-specific fusion.
_PAIR = types.SimpleNamespace(mode=None, jobs={})


@contextlib.contextmanager
def pair_weight_grads(mode):
    """``mode``: "defer" (queue main-grad dW GEMMs), "merge" (pair with the queued ones; flush the rest on
    exit) or None (plain)."""
    if mode not in ("defer", "merge", None):
        raise ValueError(f"pair_weight_grads: unknown mode {mode!r}")
    prev = _PAIR.mode
    _PAIR.mode = mode
    try:
        yield
    finally:
        _PAIR.mode = prev
        if mode == "merge":
            flush_paired_weight_grads()


def flush_paired_weight_grads():
    """Run every queued dW job on its own (then its grad-ready hook)."""
    jobs = list(_PAIR.jobs.values())
    _PAIR.jobs.clear()
    for w, x2, dy2, buf, on_ready in jobs:
        _wgrad(x2, dy2, acc=buf)
        on_ready(w)


def pending_weight_grads():
    return len(_PAIR.jobs)


def _wgrad_pair(xa, dya, xb, dyb, acc):
    """acc += xa^T dya + xb^T dyb: one two-segment GEMM when the hand-written kernel takes it and wins."""
    xta, xtb = xa.t(), xb.t()
    if G.gemm_seg_supported(xta, xtb, dya, dyb):
        key = ("wgrad2", xta.shape[0], dya.shape[1], xta.shape[1] + xtb.shape[1], acc.dtype)
        scratch = []

        def _s():
            if not scratch:
                scratch.append(torch.zeros_like(acc))
            return scratch[0]
        cands = {"hip": lambda: G.gemm_seg(xta, xtb, dya, dyb, out=_s(), accumulate=True),
                 "blas": lambda: (_s().addmm_(xta, dya), _s().addmm_(xtb, dyb))}
        if G.choose(key, cands) == "hip":
            G.gemm_seg(xta, xtb, dya, dyb, out=acc, accumulate=True)
            return
    _wgrad(xa, dya, acc=acc)
    _wgrad(xb, dyb, acc=acc)


def _main_grad_wgrad(w, x2, dy2, buf, on_ready):
    mode = _PAIR.mode
    if mode is not None:
        job = _PAIR.jobs.pop(id(w), None)
        if job is not None:  # the queued half of this weight's pair (or a tied weight met twice)
            _wgrad_pair(job[1], job[2], x2, dy2, buf)
            on_ready(w)
            return
        if mode == "defer":
            _PAIR.jobs[id(w)] = (w, x2, dy2, buf, on_ready)
            return
    _wgrad(x2, dy2, acc=buf)
    on_ready(w)


def _leaf_weights(*ws):
    """Saved at forward: the parameters themselves (activation recompute hands saved tensors back detached, and
    the zero-bubble queue / main-grad buffers are keyed by the parameter object)."""
    return tuple(w if (isinstance(w, torch.Tensor) and w.requires_grad and w.is_leaf) else None for w in ws)


def _w_ident(w, leaf, needed):
    """The object gradient routing is keyed by: the parameter saved at forward (a checkpoint recompute hands the
    saved weight back as a different tensor object), else ``w`` when it is a derived weight still attached to its
    autograd chain (a cast / slice); None when it is neither — its gradient then flows back through autograd."""
    if not needed:
        return w
    if leaf is not None:
        return leaf
    return w if w.grad_fn is not None else None


def _mm_grads(x2, w, dy2, need_x, need_w, dx_hook=None, wid=_SAME):
    """dX first, then dW. ``dx_hook(dx)`` (tensor parallelism: the column-parallel layer's dX all-reduce)
    starts an asynchronous collective on dX right after its GEMM and returns a finisher, called once the
    weight-gradient GEMM has been issued — the collective runs beside the dW GEMM instead of after it.
    ``wid``: the weight's identity for deferral / main-grad routing (see _w_ident); None = return dW."""
    dx = _dgrad(dy2, w) if need_x else None
    fin = dx_hook(dx) if (dx_hook is not None and dx is not None) else None
    dw = None
    if wid is _SAME:
        wid = w
    q = getattr(_ZB, "queue", None)
    if need_w and q is not None and wid is not None:  # zero-bubble B step: the dW GEMM runs later, in a W step
        q.append((wid, x2, dy2))
        need_w = False
    if need_w and wid is None:
        dw = _wgrad(x2, dy2)
        need_w = False
    if need_w:
        w = wid
        ent = _main_grad_of(w)
        if ent is not None and ent[1].dtype == dy2.dtype:
            _, buf, on_ready = ent
            _main_grad_wgrad(w, x2, dy2, buf, on_ready)
        else:
            dw = _wgrad(x2, dy2)
    if fin is not None:
        fin()
    return dx, dw


class _GradHook(torch.autograd.Function):
    """Identity whose backward runs ``hook(grad)`` (and its finisher) — the dX hook for linears that are not
    on the HIP path."""

    @staticmethod
    def forward(ctx, x, hook):
        ctx.hook = hook
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        fin = ctx.hook(g)
        if fin is not None:
            fin()
        return g, None


class _LinearFn(torch.autograd.Function):
    """y = x W (+ b) (+ residual): one node; the residual's gradient is dY itself."""

    @staticmethod
    def forward(ctx, x, w, b, dx_hook=None, residual=None):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if residual is not None:
            y = _fwd_mm_res(x2, w, b, residual.reshape(-1, w.shape[1]).contiguous())
        else:
            y = _fwd_mm(x2, w, b)
        ctx.res_shape = None if residual is None else residual.shape
        ctx.save_for_backward(x2, w)
        ctx.w_leaf = _leaf_weights(w)[0]
        ctx.has_b = b is not None
        ctx.bias = b
        ctx.shape = shape
        ctx.dx_hook = dx_hook
        return y.view(*shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != x2.dtype:
            dy2 = dy2.to(x2.dtype)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx, dw = _mm_grads(x2, w, dy2, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.dx_hook,
                           wid=_w_ident(w, ctx.w_leaf, ctx.needs_input_grad[1]))
        db = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            mg = _vector_main_grad(ctx.bias, dy2.dtype)
            if mg is not None:  # bias gradient added straight into its .grad buffer
                colsum(dy2, acc=mg[0])
                mg[1](ctx.bias)
            else:
                db = colsum(dy2)
        if dx is not None:
            dx = dx.view(ctx.shape)
        dres = dy.reshape(ctx.res_shape) if (ctx.res_shape is not None and ctx.needs_input_grad[4]) else None
        return dx, dw, db, None, dres


class _LinearBiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dx_hook=None):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        y, h, bb = _fwd_bias_gelu(x2, w, b)
        ctx.save_for_backward(x2, w, bb, h)
        ctx.w_leaf = _leaf_weights(w)[0]
        ctx.bias = b
        ctx.shape = shape
        ctx.dx_hook = dx_hook
        return y.view(*shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w, b, h = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).to(h.dtype).contiguous()
        rows, cols = h.shape
        dh = torch.empty_like(h)
        mg = _vector_main_grad(ctx.bias, b.dtype) if ctx.needs_input_grad[2] else None
        db = mg[0] if mg is not None else torch.empty(cols, dtype=b.dtype, device=b.device)
        ws = torch.empty(256 * cols, dtype=torch.float32, device=h.device)
        L.call("pa_bias_gelu_bwd", L.ptr(h), L.ptr(b), L.ptr(dy2), L.ptr(dh), L.ptr(db), L.ptr(ws), rows, cols,
               L.dcode(h) | ((mg is not None) << 8), L.stream_ptr())
        if mg is not None:  # bias gradient added straight into its .grad buffer
            mg[1](ctx.bias)
            db = None
        dx, dw = _mm_grads(x2, w, dh, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.dx_hook,
                           wid=_w_ident(w, ctx.w_leaf, ctx.needs_input_grad[1]))
        if dx is not None:
            dx = dx.view(ctx.shape)
        return dx, dw, db, None


def _bias_gelu_bwd(h, b, dg, db_acc=None):
    """(dh, db) of y = gelu(h + b) given dg = dL/dy (one pass, pa_bias_gelu_bwd); db added into ``db_acc``."""
    rows, cols = h.shape
    dh = torch.empty_like(h)
    db = db_acc if db_acc is not None else torch.empty(cols, dtype=b.dtype, device=b.device)
    ws = torch.empty(256 * cols, dtype=torch.float32, device=h.device)
    L.call("pa_bias_gelu_bwd", L.ptr(h), L.ptr(b), L.ptr(dg), L.ptr(dh), L.ptr(db), L.ptr(ws), rows, cols,
           L.dcode(h) | ((db_acc is not None) << 8), L.stream_ptr())
    return dh, db


def _dgrad_gelu(dy2, w2, h, b1, pre_biased, db_acc=None):
    """(dh, db1) of the FFN's hidden layer: dh = (dy2 . w2^T) * gelu'(h + b1), db1 = column sums of dh (added into
    ``db_acc`` when given). When the forward stored the biased pre-activation (hand-written GEMM, ``pre_biased``)
    the GELU backward and the bias-gradient column sums can run in the data-gradient GEMM's epilogue
    (pa_gemm_bf16_dgelu: no dY.W^T round trip through HBM); timed per shape against the separate dgrad GEMM +
    pa_bias_gelu_bwd pass (ops/gemm.py choose())."""
    w2t = w2.t()
    rows, cols = h.shape

    def split(acc=None):
        return _bias_gelu_bwd(h, b1, _dgrad(dy2, w2), acc)

    if pre_biased and G.gemm_dgelu_supported(dy2, w2t, h):
        def fused(kern, acc=None):
            dh, parts = G.gemm_dgelu(dy2, w2t, h, kern)
            db = acc if acc is not None else torch.empty(cols, dtype=h.dtype, device=h.device)
            L.call("pa_fold_partials", L.ptr(parts), L.ptr(db), cols, parts.shape[0],
                   L.dcode(h) | ((acc is not None) << 8), L.stream_ptr())
            return dh, db
        key = ("dgrad_gelu", dy2.shape[0], cols, dy2.shape[1])
        cands = {"blas": split, "hip": lambda: fused(1), "hip_4w": lambda: fused(2)}
        ch = G.choose(key, cands)
        if ch != "blas":
            CALLS["dgrad_gelu_fused"] += 1
            return fused({"hip": 1, "hip_4w": 2}[ch], db_acc)
    return split(db_acc)


CALLS = {"dgrad_gelu_fused": 0, "linear_residual": 0}


class _FFNGeluFn(torch.autograd.Function):
    """y = gelu(x W1 + b1) W2 + b2 as one autograd node (the GELU'd hidden activation has exactly one consumer
    here, so its gradient can be produced already multiplied by gelu' — see _dgrad_gelu). Reference:
    incubate/nn/functional/fused_transformer.py fused_feedforward (fused_feedforward_grad kernel); saved
    tensors are the same as two separate linears (x, pre-activation, hidden activation)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, dx_hook=None):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        a, h, bb = _fwd_bias_gelu(x2, w1, b1)
        y = _fwd_mm(a, w2, b2)
        ctx.save_for_backward(x2, w1, bb, h, a, w2)
        ctx.pre_biased = bb is not b1  # hand-written forward: h holds x W1 + b1, bb is zeros
        ctx.w_leaf = _leaf_weights(w1, w2)
        ctx.b1, ctx.b2 = b1, b2
        ctx.shape = shape
        ctx.dx_hook = dx_hook
        return y.view(*shape[:-1], w2.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w1, bb, h, a, w2 = ctx.saved_tensors
        need = ctx.needs_input_grad
        dy2 = dy.reshape(-1, dy.shape[-1]).to(h.dtype).contiguous()
        db2 = None
        if ctx.b2 is not None and need[4]:
            mg = _vector_main_grad(ctx.b2, dy2.dtype)
            if mg is not None:
                colsum(dy2, acc=mg[0])
                mg[1](ctx.b2)
            else:
                db2 = colsum(dy2)
        mg1 = _vector_main_grad(ctx.b1, h.dtype) if need[2] else None
        dh, db1 = _dgrad_gelu(dy2, w2, h, bb, ctx.pre_biased, mg1[0] if mg1 is not None else None)
        if mg1 is not None:
            mg1[1](ctx.b1)
            db1 = None
        elif not need[2]:
            db1 = None
        _, dw2 = _mm_grads(a, w2, dy2, False, need[3], wid=_w_ident(w2, ctx.w_leaf[1], need[3]))
        dx, dw1 = _mm_grads(x2, w1, dh, need[0], need[1], ctx.dx_hook, wid=_w_ident(w1, ctx.w_leaf[0], need[1]))
        if dx is not None:
            dx = dx.view(ctx.shape)
        return dx, dw1, db1, dw2, db2, None


@static_op
def ffn_gelu(x, w1, b1, w2, b2=None, dx_hook=None):
    """gelu_tanh(x @ w1 + b1) @ w2 + b2 — the GPT MLP (fc1 -> GELU -> fc2) as one fused-backward op on the HIP
    path; two fused_linear calls otherwise."""
    if _hip_linear_ok(x, w1, b1) and b1 is not None and _hip_linear_ok(x, w2, b2) and w1.shape[1] == w2.shape[0]:
        return _FFNGeluFn.apply(x, w1, b1, w2, b2, dx_hook)
    return fused_linear(fused_linear(x, w1, b1, act="gelu", dx_hook=dx_hook), w2, b2)


def _hip_linear_ok(x, w, b):
    return (L.hip_enabled_for(x) and x.dtype in (torch.bfloat16, torch.float16) and w.dtype == x.dtype
            and (b is None or b.dtype == x.dtype) and w.shape[1] % 8 == 0 and w.dim() == 2)


@static_op
def fused_linear(x, w, b=None, act=None, dx_hook=None, residual=None):
    """y = act(x @ w + b) (+ residual). ``dx_hook``: see _mm_grads (runs on the input gradient in backward).
    ``residual`` (no activation): the pre-norm decoder's residual add done by the GEMM (reference
    incubate/nn/functional/fused_rms_norm.py residual=, fused_linear_param_grad_add)."""
    hip = _hip_linear_ok(x, w, b)
    if residual is not None:
        if act is not None:
            raise ValueError("fused_linear: residual= takes no activation")
        if hip and residual.dtype == x.dtype and residual.numel() == x.numel() // x.shape[-1] * w.shape[1]:
            CALLS["linear_residual"] += 1
            return _LinearFn.apply(x, w, b, dx_hook, residual)
        return fused_linear(x, w, b, dx_hook=dx_hook) + residual
    if not hip and getattr(_ZB, "route", False) and w.dim() == 2 and torch.is_grad_enabled():
        # zero-bubble forward off the HIP path: the deferrable autograd function, activation applied after
        y = _LinearFn.apply(x, w, b, dx_hook)
        if act is None:
            return y
        if act in ("gelu", "gelu_tanh", "gelu_approximate"):
            return gelu(y, approximate=True)
        if act == "gelu_erf":
            return gelu(y, approximate=False)
        if act == "relu":
            return F.relu(y)
        raise ValueError(f"unsupported activation {act}")
    if dx_hook is not None and not (hip and (act is None or (act in ("gelu", "gelu_tanh", "gelu_approximate")
                                                             and b is not None))):
        x = _GradHook.apply(x, dx_hook)  # not a HIP linear: the hook runs on the incoming gradient
        dx_hook = None
    if act is None:
        if hip:
            return _LinearFn.apply(x, w, b, dx_hook)
        if b is None:
            return torch.matmul(x, w)
        if x.dim() == 2:
            return torch.addmm(b, x, w)
        return torch.addmm(b, x.reshape(-1, x.shape[-1]), w).view(*x.shape[:-1], w.shape[-1])
    if act in ("gelu", "gelu_tanh", "gelu_approximate"):
        if hip and b is not None:
            return _LinearBiasGeluFn.apply(x, w, b, dx_hook)
        h = torch.matmul(x, w)
        if b is not None:
            return bias_gelu(h, b)
        return gelu(h, approximate=True)
    if act == "gelu_erf":
        h = fused_linear(x, w, b)
        return gelu(h, approximate=False)
    if act == "relu":
        h = fused_linear(x, w, b)
        return F.relu(h)
    raise ValueError(f"unsupported activation {act}")


# ---------------------------------------------------------------------------------------------
# Sibling linears: y_i = x @ W_i for several weights that read the same input (q / k / v, gate / up). One
# N-segmented GEMM computes every y_i (the outputs are column views of one [.., sum N_i] tensor), the data
# gradient dx = sum_i dy_i W_i^T is ONE K-segmented GEMM over the separate dy_i (no concatenated gradient and no
# accumulation adds of partial dx), and each W_i gets its own weight gradient (main-grad / pairing aware).
# Reference: the auto-parallel fuse_attention_ffn_qkv pass (auto_parallel/static/engine.py:675) fuses the
# weights into one parameter; here the parameters stay separate and only the launches are fused, so sharding /
# checkpoints / optimizer state see the original weights. The static auto-parallel engine's fuse_sibling_linears
# pass rewrites traced programs onto this op (distributed/passes/fuse_sibling_linears.py).
class _MultiLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, *ws):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        out = G.gemm_nseg(x2, list(ws))
        ctx.save_for_backward(x2, *ws)
        ctx.w_leaves = _leaf_weights(*ws)
        ctx.shape = shape
        ctx.widths = [w.shape[1] for w in ws]
        outs = out.split(ctx.widths, dim=1)
        return tuple(o.view(*shape[:-1], o.shape[1]) for o in outs)

    @staticmethod
    def backward(ctx, *dys):
        x2, *ws = ctx.saved_tensors
        dy2s = []
        for dy in dys:
            if dy is None:
                dy2s.append(None)
                continue
            dy2 = dy.reshape(-1, dy.shape[-1])
            if dy2.dtype != x2.dtype:
                dy2 = dy2.to(x2.dtype)
            dy2s.append(dy2 if dy2.is_contiguous() else dy2.contiguous())
        live = [i for i, d in enumerate(dy2s) if d is not None]
        dx = None
        if ctx.needs_input_grad[0] and live:
            As, Bs = [dy2s[i] for i in live], [ws[i].t() for i in live]
            if G.gemm_kseg_supported(As, Bs):
                dx = G.gemm_kseg(As, Bs)
            else:
                dx = _dgrad(As[0], ws[live[0]])
                for i in live[1:]:
                    dx = dx + _dgrad(dy2s[i], ws[i])
            dx = dx.view(ctx.shape)
        grads = []
        for i, w in enumerate(ws):
            if dy2s[i] is None or not ctx.needs_input_grad[1 + i]:
                grads.append(None)
                continue
            _, dw = _mm_grads(x2, w, dy2s[i], False, True, wid=_w_ident(w, ctx.w_leaves[i], True))
            grads.append(dw)
        return (dx, *grads)


@static_op
def multi_linear(x, ws):
    """[x @ W for W in ws] (no bias): one N-segmented GEMM forward, one K-segmented data-gradient GEMM backward on
    the HIP path; separate matmuls elsewhere."""
    ws = list(ws)
    if len(ws) > 1 and len(ws) <= 4 and all(_hip_linear_ok(x, w, None) for w in ws) and \
            G.gemm_nseg_supported(x.reshape(-1, x.shape[-1]), ws):
        return list(_MultiLinearFn.apply(x, *ws))
    return [fused_linear(x, w) for w in ws]


# ---------------------------------------------------------------------------------------------
# y = x @ W^T with W stored [out, in] (the tied LM head: the embedding table is [vocab, hidden]).
# forward  y  = x  . W^T : both operands K-major (the dgrad layout of an ordinary linear)
# dgrad    dx = dy . W   : B MN-major
# wgrad    dW = dy^T . x : both MN-major (dW comes out [out, in], W's own layout; no transposes)
# Each product takes the per-shape choice between the hand-written GEMM and hipBLASLt (ops/gemm.py
# choose()), so the 3 vocabulary GEMMs of a GPT step are in the same tuning table as every other GEMM.
def _nt_fwd(x2, w):
    wt = w.t()
    if G.supported(x2, wt):
        key = ("fwd_nt", x2.shape[0], w.shape[0], x2.shape[1])
        if G.choose(key, {"blas": lambda: torch.mm(x2, wt), "hip": lambda: G.gemm(x2, wt)}) == "hip":
            return G.gemm(x2, wt)
    return torch.mm(x2, wt)


def _nt_dgrad(dy2, w):
    if G.supported(dy2, w):
        key = ("dgrad_nt", dy2.shape[0], w.shape[1], dy2.shape[1])
        if G.choose(key, {"blas": lambda: torch.mm(dy2, w), "hip": lambda: G.gemm(dy2, w)}) == "hip":
            return G.gemm(dy2, w)
    return torch.mm(dy2, w)


def _nt_wgrad(dy2, x2):
    dyt = dy2.t()
    if G.supported(dyt, x2):
        key = ("wgrad_nt", dyt.shape[0], x2.shape[1], dyt.shape[1])
        if G.choose(key, {"blas": lambda: torch.mm(dyt, x2), "hip": lambda: G.gemm(dyt, x2)}) == "hip":
            return G.gemm(dyt, x2)
    return torch.mm(dyt, x2)


class _LinearNTFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        ctx.save_for_backward(x2, w)
        ctx.shape = shape
        return _nt_fwd(x2, w).view(*shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != x2.dtype:
            dy2 = dy2.to(x2.dtype)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = _nt_dgrad(dy2, w).view(ctx.shape) if ctx.needs_input_grad[0] else None
        dw = _nt_wgrad(dy2, x2) if ctx.needs_input_grad[1] else None
        return dx, dw


@static_op
def linear_nt(x, w):
    """x @ w.T for w stored [out, in] (LM head over a tied embedding table)."""
    if _hip_linear_ok(x, w.t(), None):
        return _LinearNTFn.apply(x, w)
    return torch.matmul(x, w.t())
