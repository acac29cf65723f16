"""NHWC convolutions on the hand-written MFMA GEMM: 1x1 (forward and both gradients as GEMMs) and
KxK implicit-GEMM forward.

Reference: paddle/phi/kernels/gpu/conv_kernel.cu / conv_grad_kernel.cu (cuDNN). In NHWC a 1x1 convolution
is a plain GEMM over the N*H*W pixel rows — no im2col:
  forward  Y[P, Cout] = X[P, Cin] . W^T       (W [Cout, Cin] is the K-major B operand)
  dgrad    dX[P, Cin] = dY[P, Cout] . W       (MN-major B)
  wgrad    dW[Cout, Cin] = dY^T . X            (both operands MN-major, K = P split over workgroups)
A stride-s 1x1 convolution subsamples X first (and scatters dX back). ResNet-50 has 16 such layers
(bottleneck conv1/conv3 + the projection shortcuts). Each shape is timed once against the MIOpen path
(forward + both gradients) and the faster one is kept (ops/gemm.py choose()).

KxK (3x3, 7x7 with C % 64 == 0) forward: implicit GEMM on the 3-stage kernel (csrc/kernels/gemm.hip
pa_conv2d_nhwc_fwd): every 64-deep K tile is one filter tap x 64 channels, so an A row is a contiguous
128-byte channel slice of a shifted pixel, fetched straight to LDS by glds (taps in the padding read a
zero page); the filter in channels-last [Cout, KH, KW, C] is the K-major B operand. Gradients use MIOpen.
"""
from __future__ import annotations

import torch

from . import _loader as L
from . import _conv_bn as _CB
from . import gemm as G


class ResidualGradSink:
    """Hand-off of a residual-branch gradient between two ops of one ResNet bottleneck (identity shortcut):
    the block's last BN (which adds the block input x as its residual) writes d(residual) here instead of
    returning it to autograd, and the block's first 1x1 conv — the other consumer of x — accumulates its data
    gradient onto it in the GEMM epilogue (kEpiAccum) and returns the sum as dx. That removes the separate
    elementwise add autograd would run to sum the two gradients of x (one read + one write of an activation
    per block). ``armed`` is set only when the conv really ran the hand-written GEMM path."""

    def __init__(self):
        self.armed = False
        self.dres = None
        self.consumed = False  # the consuming conv ran before any producer (producers then return dx normally)


_SINK = [None]
_PRODUCER = [None]


class residual_grad_producer:
    """``with residual_grad_producer(sink): identity = downsample(x)`` — projection-shortcut blocks: the
    shortcut's convolution hands its data gradient to ``sink`` (returning none to autograd) and the block's first
    1x1 conv, the other consumer of x, adds it in its GEMM epilogue, so autograd never sums x's two gradients with
    a separate elementwise add. Order-safe: if the consumer already ran, the producer returns dx normally."""

    def __init__(self, sink):
        self.sink = sink

    def __enter__(self):
        _PRODUCER[0] = self.sink if (self.sink is not None and self.sink.armed) else None
        return self.sink

    def __exit__(self, *exc):
        _PRODUCER[0] = None
        return False


class residual_grad_sink:
    """``with residual_grad_sink() as s: y = conv1(x)`` — a 1x1 conv on the HIP path inside the block arms s."""

    def __enter__(self):
        self.sink = ResidualGradSink()
        _SINK[0] = self.sink
        return self.sink

    def __exit__(self, *exc):
        _SINK[0] = None
        return False


def _splits(M, N, K):
    return G.pick_splits(M, N, K, bn=G._pick_bn(M, N, False))


def _wgrad_1x1(a, b, splits, dtype):
    """dW = dY^T . X of a 1x1 convolution (K = every pixel of the batch): split-K on the generic kernel or on the
    ping-pong 256x256 kernel, whichever the per-shape timing picks (the ping-pong form needs >= 256-wide outputs to
    pay off)."""
    M, N, K = a.shape[0], b.shape[1], a.shape[1]
    sp = G.pp_splits(M, N, K)
    if M >= 256 and N >= 256 and G.gemm_pp_splitk_ok(a, b, sp):
        ch = G.choose(("wgrad1x1", M, N, K), {"hip": lambda: G.gemm_splitk(a, b, splits, out_dtype=dtype),
                                              "hip_pp": lambda: G.gemm_pp_splitk(a, b, sp, dtype)})
        if ch == "hip_pp":
            return G.gemm_pp_splitk(a, b, sp, dtype)
    return G.gemm_splitk(a, b, splits, out_dtype=dtype)


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, sink=None):
        ctx.sink = sink
        N, H, W, Cin = x.shape
        Cout = w.shape[0]
        xs = x[:, ::stride, ::stride, :].contiguous() if stride > 1 else x
        Ho, Wo = xs.shape[1], xs.shape[2]
        x2 = xs.reshape(-1, Cin)
        w2 = w.reshape(Cout, Cin)
        y2 = G.gemm(x2, w2.t(), bias=b)
        ctx.save_for_backward(x2, w2)
        ctx.meta = (N, H, W, Cin, Cout, Ho, Wo, stride, b is not None)
        return y2.view(N, Ho, Wo, Cout)

    @staticmethod
    def backward(ctx, dy):
        x2, w2 = ctx.saved_tensors
        N, H, W, Cin, Cout, Ho, Wo, stride, has_b = ctx.meta
        dy2 = dy.reshape(-1, Cout)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = db = None
        sink = ctx.sink
        if ctx.needs_input_grad[0]:
            if sink is not None and sink.dres is not None and stride == 1:
                # dx = d(residual) + dy . W in one epilogue (see ResidualGradSink)
                acc = sink.dres
                sink.dres = None
                dx2 = G.gemm(dy2, w2, out=acc.view(-1, Cin), accumulate=True)
            else:
                dx2 = G.gemm(dy2, w2)
            dx = dx2.view(N, Ho, Wo, Cin)
            if stride > 1:
                full = torch.zeros(N, H, W, Cin, dtype=dx.dtype, device=dx.device)
                full[:, ::stride, ::stride, :] = dx
                dx = full
        if ctx.needs_input_grad[1]:
            P = dy2.shape[0]
            if P % 64 == 0:
                dw = _wgrad_1x1(dy2.t(), x2, _splits(Cout, Cin, P), w2.dtype)
            else:  # pixel count not a multiple of the 64-deep K tile
                dw = torch.mm(dy2.t(), x2)
            dw = dw.view(Cout, Cin, 1, 1)
        if has_b and ctx.needs_input_grad[2]:
            db = dy2.float().sum(0).to(dy2.dtype)
        return dx, dw, db, None, None


def eligible(x_nhwc, w, groups, padding_is_zero, dilation_ok=True):
    """Shape / layout conditions of the GEMM path for a 2-D NHWC convolution."""
    if not (x_nhwc.is_cuda and x_nhwc.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    if x_nhwc.dim() != 4 or w.dim() != 4 or tuple(w.shape[2:]) != (1, 1) or groups != 1 or not padding_is_zero:
        return False
    if not x_nhwc.is_contiguous() or not L.has("pa_gemm_bf16") or not L.hip_enabled_for(x_nhwc):
        return False
    cin, cout = x_nhwc.shape[3], w.shape[0]
    return cin % 64 == 0 and cout % 64 == 0 and x_nhwc.numel() > 0  # K of forward / data-gradient GEMMs


def conv1x1_nhwc(x, w, b, stride, fallback):
    """x: [N, H, W, Cin] contiguous bf16; w: [Cout, Cin, 1, 1]; ``fallback()`` runs the MIOpen path and
    returns the NHWC result. Picks the faster per shape (forward + backward timed once)."""
    key = ("conv1x1", tuple(x.shape), w.shape[0], stride, b is not None, x.requires_grad or w.requires_grad)

    sink = _SINK[0] if stride == 1 else None

    def hip():
        if sink is not None:
            sink.armed = True
        return _Conv1x1.apply(x, w, b, stride, sink)

    def _fb_bench(fn):
        def run():
            xx = x.detach().requires_grad_(True)
            ww = w.detach().requires_grad_(True)
            with torch.enable_grad():
                y = fn(xx, ww)
                y.backward(torch.ones_like(y))
        return run
    if not G.known(key) and not G._capturing() and L.flag("FLAGS_gemm_backend", "auto") == "auto":
        G.choose(key, {"hip": _fb_bench(lambda xx, ww: _Conv1x1.apply(xx, ww, b, stride)),
                       "blas": _fb_bench(lambda xx, ww: fallback(xx, ww))})
    ch = G.choose(key, {"hip": hip, "blas": lambda: None})
    if ch == "hip":
        return hip()
    return None


_ZERO = {}


def _zero_page(dev):
    z = _ZERO.get(dev)
    if z is None:
        z = _ZERO[dev] = torch.zeros(128, dtype=torch.bfloat16, device=dev)
    return z


def _ph_pw(pad):
    """(pad_h, pad_w) of an int or (h, w) padding (1-D convolutions run as 1 x K with padding (0, p))."""
    return (pad, pad) if isinstance(pad, int) else (int(pad[0]), int(pad[1]))


def _implicit_fwd(x, wk, b, N, H, W, C, Cout, KH, KW, stride, pad, dil):
    ph, pw = _ph_pw(pad)
    Ho = (H + 2 * ph - dil * (KH - 1) - 1) // stride + 1
    Wo = (W + 2 * pw - dil * (KW - 1) - 1) // stride + 1
    out = torch.empty(N, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    L.call("pa_conv2d_nhwc_fwd", L.ptr(x), L.ptr(wk), L.ptr(b), L.ptr(out), L.ptr(_zero_page(x.device)), N, H, W,
           C, Cout, KH, KW, stride, ph, pw, dil, Ho, Wo, L.stream_ptr())
    return out


def _wgrad_splits(P, M, N, bn=128, cus=256, max_ws_bytes=256 << 20):
    """Split-K factor for the implicit weight gradient: about two workgroups per CU, K slices a multiple of
    the 64-pixel tile, fp32 slabs within the workspace budget."""
    tiles = -(-M // 256) * -(-N // bn)
    s = 1
    while (tiles * s * 2 <= 2 * cus and P % (64 * s * 2) == 0 and (s * 2) * M * N * 4 <= max_ws_bytes):
        s *= 2
    return s


def _implicit_wgrad(x, dy, w, N, H, W, C, Cout, KH, KW, stride, pad, dil, Ho, Wo):
    """dW [Cout, C, KH, KW] = im2col(x)^T . dy as a split-K implicit GEMM (csrc/kernels/gemm.hip
    pa_conv2d_nhwc_wgrad: the im2col rows are gathered per pixel and tap on the fly, no im2col buffer)."""
    M = KH * KW * C
    bn = 256 if Cout % 256 == 0 else (64 if Cout <= 64 else 128)
    splits = _wgrad_splits(N * Ho * Wo, M, Cout, bn)
    ws = torch.empty(splits, M, Cout, dtype=torch.float32, device=x.device)
    ph, pw = _ph_pw(pad)
    L.call("pa_conv2d_nhwc_wgrad", L.ptr(x), L.ptr(dy), L.ptr(ws), L.ptr(_zero_page(x.device)), N, H, W, C, Cout, KH,
           KW, stride, ph, pw, dil, Ho, Wo, splits, bn, L.stream_ptr())
    dwt = G.reduce_slabs(ws, w.dtype)
    return dwt.view(KH, KW, C, Cout).permute(3, 2, 0, 1).to(w.dtype).contiguous(memory_format=torch.channels_last) \
        if w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous() else \
        dwt.view(KH, KW, C, Cout).permute(3, 2, 0, 1).to(w.dtype).contiguous()


class _ConvImplicit(torch.autograd.Function):
    """Forward: implicit GEMM. Data gradient (stride 1, no dilation): the same implicit GEMM over dY with
    the filter flipped and its channel axes swapped (W'[c, kh, kw, co] = W[co, KH-1-kh, KW-1-kw, c]),
    padding KH-1-pad. Weight gradient: split-K implicit GEMM gathering the im2col rows of x (any stride /
    padding / dilation). The strided data gradient: MIOpen."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil):
        N, H, W, C = x.shape
        Cout, _, KH, KW = w.shape
        wk = w.permute(0, 2, 3, 1)
        if not wk.is_contiguous():
            wk = wk.contiguous()
        out = _implicit_fwd(x, wk, b, N, H, W, C, Cout, KH, KW, stride, pad, dil)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, dil, b is not None)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, dil, has_b = ctx.cfg
        N, H, W, C = x.shape
        Cout, _, KH, KW = w.shape
        dy = dy.contiguous()
        dx = None
        own_dx = (ctx.needs_input_grad[0] and stride == 1 and dil == 1 and Cout % 64 == 0 and C % 8 == 0
                  and 2 * pad <= KH - 1 + pad and KH == KW)
        if own_dx:
            # [C, KH, KW, Cout] flipped filter (K-major B operand of the transposed convolution)
            wt = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()
            Ho, Wo = dy.shape[1], dy.shape[2]
            dx = _implicit_fwd(dy, wt, None, N, Ho, Wo, Cout, C, KH, KW, 1, KH - 1 - pad, 1)
        Ho, Wo = dy.shape[1], dy.shape[2]
        P = N * Ho * Wo
        own_dw = (ctx.needs_input_grad[1] and L.has("pa_conv2d_nhwc_wgrad") and C % 8 == 0 and Cout % 8 == 0
                  and P % 64 == 0)
        if own_dw:
            # per-shape choice against MIOpen's weight gradient (profiles/conv_wgrad_vs_miopen.log)
            def _miopen_dw():
                return torch.ops.aten.convolution_backward(
                    dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w, None, [stride] * 2, [pad] * 2, [dil] * 2,
                    False, [0, 0], 1, [False, True, False])[1]
            key = ("convw", tuple(x.shape), tuple(w.shape), stride, pad, dil)
            own_dw = G.choose(key, {"hip": lambda: _implicit_wgrad(x, dy, w, N, H, W, C, Cout, KH, KW, stride, pad,
                                                                   dil, Ho, Wo),
                                    "blas": _miopen_dw}) == "hip"
        gw = None
        if own_dw:
            gw = _implicit_wgrad(x, dy, w, N, H, W, C, Cout, KH, KW, stride, pad, dil, Ho, Wo)
        mask = [ctx.needs_input_grad[0] and not own_dx, ctx.needs_input_grad[1] and not own_dw,
                has_b and ctx.needs_input_grad[2]]
        gb = None
        if any(mask):
            xc = x.permute(0, 3, 1, 2)
            dyc = dy.permute(0, 3, 1, 2)
            wc = w if w.is_contiguous(memory_format=torch.channels_last) else \
                w.contiguous(memory_format=torch.channels_last)
            gi, gw2, gb = torch.ops.aten.convolution_backward(dyc, xc, wc, [w.shape[0]] if has_b else None,
                                                              [stride] * 2, [pad] * 2, [dil] * 2, False, [0, 0], 1, mask)
            if gi is not None:
                dx = gi.permute(0, 2, 3, 1)
            if gw2 is not None:
                gw = gw2
        return dx, gw, gb, None, None, None


# ---------------------------------------------------------------------------------------------
# Per-direction backend choice. A convolution is three products (forward, data gradient, weight gradient)
# and the hand-written kernel and MIOpen win different ones on the same layer: e.g. on the 56x56 stage of
# ResNet-50 our 1x1 data gradient (a K=64 GEMM) beats MIOpen while its forward does not. _ConvNHWC picks
# each direction separately (keys convf / convd / convw, timed once on first use like every GEMM key,
# tools/bench_conv_dir.py), so a layer never pays for the losing direction of the winning side.
def _mi_weight(w):
    return w if w.is_contiguous(memory_format=torch.channels_last) else w.contiguous(memory_format=torch.channels_last)


def _mi_fwd(x, w, b, stride, pad, dil):
    y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), _mi_weight(w), b, stride, pad, dil)
    y = y.permute(0, 2, 3, 1)
    return y if y.is_contiguous() else y.contiguous()


def _mi_bwd(x, w, dy, stride, pad, dil, mask):
    pad = _ph_pw(pad)
    gi, gw, _ = torch.ops.aten.convolution_backward(dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), _mi_weight(w),
                                                    None, [stride] * 2, list(pad), [dil] * 2, False, [0, 0], 1,
                                                    mask + [False])
    if gi is not None:
        gi = gi.permute(0, 2, 3, 1)
        gi = gi if gi.is_contiguous() else gi.contiguous()
    return gi, gw


def _skinny_conv(x, wk, b, N, H, W, C, Cout, KH, KW, stride, pad):
    """KxK convolution on the skinny implicit-GEMM kernel (csrc/kernels/gemm_skinny.hip pa_conv_skinny);
    wk: filter [Cout, KH, KW, C] contiguous."""
    Ho = (H + 2 * pad - KH) // stride + 1
    Wo = (W + 2 * pad - KW) // stride + 1
    out = torch.empty(N, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    L.call("pa_conv_skinny", L.ptr(x), L.ptr(wk), L.ptr(b), L.ptr(out), L.ptr(_zero_page(x.device)), N, H, W, C, Cout,
           KH, KW, stride, pad, Ho, Wo, L.stream_ptr())
    return out


def _skinny_ok(x, w, stride, dgrad, pad=0, dil=1):
    """Products the memory-bound skinny kernels take: 1x1 (ops/gemm.py gemm_skinny: N, K in {32..256}, tall M)
    and KxK (pa_conv_skinny: C = Cout = 64, 3x3; the data gradient only at stride 1)."""
    if not isinstance(pad, int):
        return False
    C, Cout = x.shape[3], w.shape[0]
    if not (w.shape[2] == 1 and w.shape[3] == 1):
        if not L.has("pa_conv_skinny") or dil != 1 or (dgrad and stride != 1) or x.numel() * 2 >= (1 << 31) - (1 << 21):
            return False
        ci, co = (Cout, C) if dgrad else (C, Cout)
        return bool(L.lib().pa_conv_skinny_ok(ci, co, w.shape[2], w.shape[3]))
    if not L.has("pa_gemm_skinny"):
        return False
    M = x.shape[0] * (-(-x.shape[1] // stride)) * (-(-x.shape[2] // stride))
    n, k = (C, Cout) if dgrad else (Cout, C)
    return M >= 1024 and bool(L.lib().pa_gemm_skinny_ok(n, k))


def _skinny_stats_ok(x, w, stride, pad, dil):
    """The skinny kernels with a statistics epilogue: 1x1 with Cout <= 128, the 3x3 stride-1 pad-1 halo kernel."""
    Cout, _, KH, KW = w.shape
    if KH == 1 and KW == 1:
        return L.has("pa_gemm_skinny_stats") and Cout <= 128
    return L.has("pa_conv_skinny_stats") and stride == 1 and pad == 1 and dil == 1


def _own_fwd_stats(x, w, b, stride, pad, dil, skinny=False, bn=None):
    """The hand-written forward that also writes the following BN's partials (conv -> BN fusion, ops/_conv_bn.py):
    (y, (stats, chunks)). bn: GEMM tile width of a 1x1 convolution (160 / 128)."""
    N, H, W, C = x.shape
    Cout, _, KH, KW = w.shape
    if KH == 1 and KW == 1:
        xs = x[:, ::stride, ::stride, :].contiguous() if stride > 1 else x
        if skinny:
            y2, stats, chunks = G.gemm_skinny_bn_stats(xs.reshape(-1, C), w.reshape(Cout, C).t(), bias=b)
        else:
            y2, stats, chunks = G.gemm_bn_stats(xs.reshape(-1, C), w.reshape(Cout, C).t(), bias=b, bn=bn)
        return y2.view(N, xs.shape[1], xs.shape[2], Cout), (stats, chunks)
    wk = w.permute(0, 2, 3, 1)
    if not wk.is_contiguous():
        wk = wk.contiguous()
    if skinny:
        out = torch.empty(N, H, W, Cout, dtype=x.dtype, device=x.device)
        chunks = int(L.lib().pa_conv_skinny_stats_chunks(N, H, W))
        stats = torch.empty(2 * chunks * Cout, dtype=torch.float32, device=x.device)
        L.call("pa_conv_skinny_stats", L.ptr(x), L.ptr(wk), L.ptr(b), L.ptr(out), L.ptr(_zero_page(x.device)), N, H, W,
               L.ptr(stats), L.stream_ptr())
        return out, (stats, chunks)
    ph, pw = _ph_pw(pad)
    Ho = (H + 2 * ph - dil * (KH - 1) - 1) // stride + 1
    Wo = (W + 2 * pw - dil * (KW - 1) - 1) // stride + 1
    out = torch.empty(N, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    chunks = int(L.lib().pa_gemm_stats_chunks(N * Ho * Wo, 160))
    stats = torch.empty(2 * chunks * Cout, dtype=torch.float32, device=x.device)
    L.call("pa_conv2d_nhwc_fwd_stats", L.ptr(x), L.ptr(wk), L.ptr(b), L.ptr(out), L.ptr(_zero_page(x.device)), N, H,
           W, C, Cout, KH, KW, stride, ph, pw, dil, Ho, Wo, L.ptr(stats), L.stream_ptr())
    return out, (stats, chunks)


def _own_fwd(x, w, b, stride, pad, dil, skinny=False):
    N, H, W, C = x.shape
    Cout, _, KH, KW = w.shape
    if KH == 1 and KW == 1:
        xs = x[:, ::stride, ::stride, :].contiguous() if stride > 1 else x
        if skinny:
            y2 = G.gemm_skinny(xs.reshape(-1, C), w.reshape(Cout, C).t(), bias=b)
        else:
            y2 = G.gemm(xs.reshape(-1, C), w.reshape(Cout, C).t(), bias=b)
        return y2.view(N, xs.shape[1], xs.shape[2], Cout)
    wk = w.permute(0, 2, 3, 1)
    if not wk.is_contiguous():
        wk = wk.contiguous()
    if skinny:
        return _skinny_conv(x, wk, b, N, H, W, C, Cout, KH, KW, stride, pad)
    return _implicit_fwd(x, wk, b, N, H, W, C, Cout, KH, KW, stride, pad, dil)


def _own_dgrad_ok(x, w, stride, pad, dil):
    C, (Cout, _, KH, KW) = x.shape[3], w.shape
    if not isinstance(pad, int):
        return False  # asymmetric (1-D) padding: MIOpen
    if KH == 1 and KW == 1:
        return True
    return stride == 1 and dil == 1 and Cout % 64 == 0 and C % 8 == 0 and 2 * pad <= KH - 1 + pad and KH == KW


def _own_dgrad(x, w, dy, stride, pad, dil, acc=None, skinny=False):
    """dX on the hand-written kernels; ``acc`` (1x1, stride 1): NHWC gradient dX is added onto in the epilogue."""
    N, H, W, C = x.shape
    Cout, _, KH, KW = w.shape
    if KH == 1 and KW == 1:
        dy2 = dy.reshape(-1, Cout)
        w2 = w.reshape(Cout, C)
        mm = G.gemm_skinny if skinny else G.gemm
        if acc is not None and stride == 1:
            return mm(dy2, w2, out=acc.view(-1, C), accumulate=True).view(N, H, W, C)
        dx = mm(dy2, w2).view(N, dy.shape[1], dy.shape[2], C)
        if stride > 1:
            full = torch.zeros(N, H, W, C, dtype=dx.dtype, device=dx.device)
            full[:, ::stride, ::stride, :] = dx
            dx = full
        return dx
    # transposed convolution = convolution of dY with the flipped, in/out-swapped filter [C, KH, KW, Cout]
    wt = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()
    if skinny:
        return _skinny_conv(dy, wt, None, N, dy.shape[1], dy.shape[2], Cout, C, KH, KW, 1, KH - 1 - pad)
    return _implicit_fwd(dy, wt, None, N, dy.shape[1], dy.shape[2], Cout, C, KH, KW, 1, KH - 1 - pad, 1)


def _bnbwd_ok(x, w, stride, pad, dil):
    """Data gradients with the BN-backward statistics epilogue: stride-1 1x1 (GEMM) and stride-1 KxK
    (implicit GEMM of the flipped filter) on the hand-written kernels."""
    if not (L.has("pa_gemm_bf16_bnbwd") and stride == 1 and _own_dgrad_ok(x, w, stride, pad, dil)):
        return False
    return x.shape[3] % 8 == 0 and w.shape[1] == x.shape[3]


def _own_dgrad_bnbwd(x, w, dy, pad, src):
    """dX of a stride-1 convolution whose input is a relu BN's output, with the BN-backward partials of dX
    ([sum dyp, sum dyp * (x_bn - mean)]) written by the epilogue: (dX, (stats, chunks))."""
    bx, mean, ss = src
    N, H, W, C = x.shape
    Cout, _, KH, KW = w.shape
    if KH == 1 and KW == 1:
        dy2 = dy.reshape(-1, Cout)
        w2 = w.reshape(Cout, C)
        M = dy2.shape[0]
        lda, ak = G._layout(dy2, 0)
        ldb, bk = G._layout(w2, 1)
        bn = 160 if bk else (256 if G._pick_bn(M, C, bk) == 256 else 128)
        chunks = int(L.lib().pa_gemm_stats_chunks(M, bn))
        dx = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
        stats = torch.empty(2 * chunks * C, dtype=torch.float32, device=dy.device)
        L.call("pa_gemm_bf16_bnbwd", L.ptr(dy2), L.ptr(w2), L.ptr(dx), M, C, Cout, lda, ldb, C, int(ak), int(bk), bn,
               L.ptr(bx), L.ptr(ss), L.ptr(mean), L.ptr(stats), L.stream_ptr())
        return dx, (stats, chunks)
    wt = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()
    Ho, Wo = dy.shape[1], dy.shape[2]
    pd = KH - 1 - pad
    Hx = (Ho + 2 * pd - (KH - 1) - 1) + 1
    Wx = (Wo + 2 * pd - (KW - 1) - 1) + 1
    dx = torch.empty(N, Hx, Wx, C, dtype=dy.dtype, device=dy.device)
    chunks = int(L.lib().pa_gemm_stats_chunks(N * Hx * Wx, 160))
    stats = torch.empty(2 * chunks * C, dtype=torch.float32, device=dy.device)
    L.call("pa_conv2d_nhwc_fwd_bnbwd", L.ptr(dy), L.ptr(wt), L.ptr(dx), L.ptr(_zero_page(dy.device)), N, Ho, Wo, Cout,
           C, KH, KW, 1, pd, pd, 1, Hx, Wx, L.ptr(bx), L.ptr(ss), L.ptr(mean), L.ptr(stats), L.stream_ptr())
    return dx, (stats, chunks)


def _own_wgrad_ok(x, w, dy):
    C, Cout = x.shape[3], w.shape[0]
    P = dy.shape[0] * dy.shape[1] * dy.shape[2]
    if w.shape[2] == 1 and w.shape[3] == 1:
        return P % 64 == 0
    return L.has("pa_conv2d_nhwc_wgrad") and C % 8 == 0 and Cout % 8 == 0 and P % 64 == 0


def _own_wgrad(x, w, dy, stride, pad, dil):
    N, H, W, C = x.shape
    Cout, _, KH, KW = w.shape
    if KH == 1 and KW == 1:
        xs = x[:, ::stride, ::stride, :].contiguous() if stride > 1 else x
        x2 = xs.reshape(-1, C)
        dy2 = dy.reshape(-1, Cout)
        dw = G.gemm_splitk(dy2.t(), x2, _splits(Cout, C, dy2.shape[0]), out_dtype=w.dtype)
        return dw.view(Cout, C, 1, 1)
    return _implicit_wgrad(x, dy, w, N, H, W, C, Cout, KH, KW, stride, pad, dil, dy.shape[1], dy.shape[2])


def _skinny_wgrad_ok(x, w, dy, stride, pad, dil):
    """3x3 stride-1 pad-1 C = Cout = 64 weight gradient on the halo-tile kernel (pa_conv_skinny_wgrad)."""
    return (L.has("pa_conv_skinny_wgrad") and tuple(w.shape) == (64, 64, 3, 3) and x.shape[3] == 64 and stride == 1
            and pad == 1 and dil == 1 and tuple(dy.shape[1:3]) == tuple(x.shape[1:3]))


def _skinny_wgrad(x, dy, w):
    N, H, W, C = x.shape
    npieces = N * H * (-(-W // 32))
    splits = max(1, min(256, npieces))
    ws = torch.empty(splits, 64 * 9 * 64, dtype=torch.float32, device=x.device)
    L.call("pa_conv_skinny_wgrad", L.ptr(x), L.ptr(dy), L.ptr(_zero_page(x.device)), L.ptr(ws), N, H, W, C, 64,
           splits, L.stream_ptr())
    dw = G.reduce_slabs(ws.view(splits, 1, -1), w.dtype).view(64, 3, 3, 64).permute(0, 3, 1, 2).to(w.dtype)
    return dw.contiguous(memory_format=torch.channels_last) \
        if w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous() else dw.contiguous()


def _pick(key, own, mi, skinny=None, mm=None, extra=None):
    """'hip' | 'skinny' | 'mm' | 'blas' for one direction (ops/gemm.py choose(): timed once, persisted). 'skinny'
    is the memory-bound kernel, offered when the shape fits it; 'mm' a 1x1 product as a hipBLASLt GEMM. Timed
    with cold caches: in a training step every activation streams from HBM, while a repeated call would find a
    100 MB input in the 256 MB MALL and favour the kernels that profit most from that."""
    if L.flag("FLAGS_gemm_backend", "auto") != "auto":
        return G.choose(key, {"hip": None, "blas": None})
    cands = {"hip": own, "blas": mi}
    if skinny is not None:
        cands["skinny"] = skinny
    if mm is not None:
        cands["mm"] = mm
    cands.update(extra or {})
    return G.choose(key, cands, cold=True)


def _mm_fwd(x, w, b, stride):
    """1x1 forward as a hipBLASLt GEMM (the 'mm' candidate)."""
    N, C, Cout = x.shape[0], x.shape[3], w.shape[0]
    xs = x[:, ::stride, ::stride, :].contiguous() if stride > 1 else x
    x2 = xs.reshape(-1, C)
    w2 = w.reshape(Cout, C)
    y2 = torch.mm(x2, w2.t()) if b is None else torch.addmm(b, x2, w2.t())
    return y2.view(N, xs.shape[1], xs.shape[2], Cout)


def _mm_dgrad(x, w, dy, stride, acc=None):
    N, H, W, C = x.shape
    Cout = w.shape[0]
    dy2 = dy.reshape(-1, Cout)
    w2 = w.reshape(Cout, C)
    if acc is not None and stride == 1:
        return acc.view(-1, C).addmm_(dy2, w2).view(N, H, W, C)
    dx = torch.mm(dy2, w2).view(N, dy.shape[1], dy.shape[2], C)
    if stride > 1:
        full = torch.zeros(N, H, W, C, dtype=dx.dtype, device=dx.device)
        full[:, ::stride, ::stride, :] = dx
        dx = full
    return dx


class _ConvNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil, sink=None, produce=None, bn_stats=False, bn_src=None):
        key = (tuple(x.shape), tuple(w.shape), stride, pad, dil)
        one = w.shape[2] == 1 and w.shape[3] == 1
        _CB._PENDING[0] = None
        sk_stats = False
        if bn_stats:
            # a training BN consumes the output: the hand-written kernels write its statistics in the epilogue;
            # the other candidates are timed with the statistics pass the BN then runs itself
            red = _CB.reduce_cost
            sk = None
            sk_stats = _skinny_ok(x, w, stride, False, pad, dil) and _skinny_stats_ok(x, w, stride, pad, dil)
            if sk_stats:
                sk = lambda: _own_fwd_stats(x, w, b, stride, pad, dil, skinny=True)  # noqa: E731
            elif _skinny_ok(x, w, stride, False, pad, dil):
                sk = lambda: red(_own_fwd(x, w, b, stride, pad, dil, skinny=True))  # noqa: E731
            # 'hipu': the hand-written kernel without the statistics epilogue (e.g. the ping-pong 256x256 GEMM
            # of a large 1x1 convolution, which has no statistics variant) plus the BN's own statistics pass
            ch = _pick(("convf",) + key + (b is not None, "bn"), lambda: _own_fwd_stats(x, w, b, stride, pad, dil),
                       lambda: red(_mi_fwd(x, w, b, stride, pad, dil)), sk,
                       (lambda: red(_mm_fwd(x, w, b, stride))) if one else None,
                       dict({"hipu": lambda: red(_own_fwd(x, w, b, stride, pad, dil))},
                            **({"hip128": lambda: _own_fwd_stats(x, w, b, stride, pad, dil, bn=128)}
                               if one and w.shape[0] <= 128 else {})))
        else:
            sk = (lambda: _own_fwd(x, w, b, stride, pad, dil, skinny=True)) \
                if _skinny_ok(x, w, stride, False, pad, dil) else None
            ch = _pick(("convf",) + key + (b is not None,), lambda: _own_fwd(x, w, b, stride, pad, dil),
                       lambda: _mi_fwd(x, w, b, stride, pad, dil), sk,
                       (lambda: _mm_fwd(x, w, b, stride)) if one else None)
        if ch == "blas":
            y = _mi_fwd(x, w, b, stride, pad, dil)
        elif ch == "mm":
            y = _mm_fwd(x, w, b, stride)
        elif ch == "hipu":
            y = _own_fwd(x, w, b, stride, pad, dil)
        elif ch == "hip128":
            y, _CB._PENDING[0] = _own_fwd_stats(x, w, b, stride, pad, dil, bn=128)
        elif ch == "hip" and bn_stats:
            y, _CB._PENDING[0] = _own_fwd_stats(x, w, b, stride, pad, dil)
        elif ch == "skinny" and bn_stats and sk_stats:
            y, _CB._PENDING[0] = _own_fwd_stats(x, w, b, stride, pad, dil, skinny=True)
        else:
            y = _own_fwd(x, w, b, stride, pad, dil, skinny=ch == "skinny")
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, dil, b is not None, key)
        ctx.sink = sink
        ctx.produce = produce
        ctx.bn_src = bn_src  # (x, mean, scale-shift) of the relu BN that produced x: fused backward statistics
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, dil, has_b, key = ctx.cfg
        dy = dy if dy.is_contiguous() else dy.contiguous()
        dres = None
        if ctx.sink is not None:
            dres, ctx.sink.dres = ctx.sink.dres, None
            if dres is None:
                ctx.sink.consumed = True
        dx = dw = db = None
        src = ctx.bn_src if dres is None and ctx.needs_input_grad[0] else None
        if src is not None and _bnbwd_ok(x, w, stride, pad, dil):
            red = _CB.reduce_cost_bwd
            sk = (lambda: red(_own_dgrad(x, w, dy, stride, pad, dil, skinny=True), src)) \
                if _skinny_ok(x, w, stride, True, pad, dil) else None
            one = w.shape[2] == 1 and w.shape[3] == 1
            ch = _pick(("convd",) + key + ("bnbwd",), lambda: _own_dgrad_bnbwd(x, w, dy, pad, src),
                       lambda: red(_mi_bwd(x, w, dy, stride, pad, dil, [True, False])[0], src), sk,
                       (lambda: red(_mm_dgrad(x, w, dy, stride), src)) if one else None,
                       {"hipu": lambda: red(_own_dgrad(x, w, dy, stride, pad, dil), src)})
            if ch == "hip":
                dx, (stats, chunks) = _own_dgrad_bnbwd(x, w, dy, pad, src)
                _CB.put_bwd(dx, stats, chunks, src[0])
            elif ch == "hipu":
                dx = _own_dgrad(x, w, dy, stride, pad, dil)
            elif ch == "skinny":
                dx = _own_dgrad(x, w, dy, stride, pad, dil, skinny=True)
            elif ch == "mm":
                dx = _mm_dgrad(x, w, dy, stride)
            else:
                dx = _mi_bwd(x, w, dy, stride, pad, dil, [True, False])[0]
        elif ctx.needs_input_grad[0]:
            ch = "blas"
            if _own_dgrad_ok(x, w, stride, pad, dil):
                sk = (lambda: _own_dgrad(x, w, dy, stride, pad, dil, skinny=True)) \
                    if _skinny_ok(x, w, stride, True, pad, dil) else None
                one = w.shape[2] == 1 and w.shape[3] == 1
                ch = _pick(("convd",) + key, lambda: _own_dgrad(x, w, dy, stride, pad, dil),
                           lambda: _mi_bwd(x, w, dy, stride, pad, dil, [True, False]), sk,
                           (lambda: _mm_dgrad(x, w, dy, stride)) if one else None)
            if ch == "mm":
                dx = _mm_dgrad(x, w, dy, stride, acc=dres)
                if dres is not None and stride != 1:
                    dx = dx + dres
            elif ch != "blas":
                dx = _own_dgrad(x, w, dy, stride, pad, dil, acc=dres, skinny=ch == "skinny")
                if dres is not None and not (w.shape[2] == 1 and w.shape[3] == 1 and stride == 1):
                    dx = dx + dres
            else:
                dx = _mi_bwd(x, w, dy, stride, pad, dil, [True, False])[0]
                if dres is not None:
                    dx = dx.add_(dres)
        elif dres is not None:
            dx = dres
        if ctx.needs_input_grad[1]:
            ch = "blas"
            if _own_wgrad_ok(x, w, dy):
                sk = (lambda: _skinny_wgrad(x, dy, w)) if _skinny_wgrad_ok(x, w, dy, stride, pad, dil) else None
                ch = _pick(("convw",) + key, lambda: _own_wgrad(x, w, dy, stride, pad, dil),
                           lambda: _mi_bwd(x, w, dy, stride, pad, dil, [False, True]), sk)
            if ch == "skinny":
                dw = _skinny_wgrad(x, dy, w)
            elif ch == "hip":
                dw = _own_wgrad(x, w, dy, stride, pad, dil)
            else:
                dw = _mi_bwd(x, w, dy, stride, pad, dil, [False, True])[1]
            if dw.dtype != w.dtype:
                dw = dw.to(w.dtype)
        if has_b and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, dy.shape[-1]).float().sum(0).to(dy.dtype)
        prod = ctx.produce
        if prod is not None and dx is not None and not prod.consumed:
            dx = dx if dx.is_contiguous() else dx.contiguous()
            prod.dres = dx if prod.dres is None else prod.dres.add_(dx)
            dx = None  # the block's first conv adds it (residual_grad_producer)
        return dx, dw, db, None, None, None, None, None, None, None


def conv2d_nhwc(x, w, b, stride, pad, dil, bn_stats=None):
    """NHWC 2-D convolution (groups 1; ``pad`` an int or a per-dimension (ph, pw) pair) with each of its three
    products on the hand-written kernel or MIOpen, whichever measured faster for the shape. A stride-1 1x1
    convolution inside ``residual_grad_sink()`` takes over the block's residual gradient (ResidualGradSink).
    ``bn_stats``: True when the caller knows a training BN consumes the output (fused units), None to learn it
    (ops/_conv_bn.py)."""
    if not isinstance(pad, int):
        pad = int(pad[0]) if pad[0] == pad[1] else (int(pad[0]), int(pad[1]))
    sink = _SINK[0] if (w.shape[2] == 1 and w.shape[3] == 1 and stride == 1) else None
    if sink is not None:
        sink.armed = True
    produce, _PRODUCER[0] = _PRODUCER[0], None
    if produce is not None and produce is sink:
        produce = None
    key = (tuple(x.shape), tuple(w.shape), stride, pad, dil)
    want = _CB.wanted(key) if bn_stats is None else (bool(bn_stats) and torch.is_grad_enabled() and _CB.enabled())
    src = _CB.bn_source(x) if torch.is_grad_enabled() else None
    y = _ConvNHWC.apply(x, w, b, stride, pad, dil, sink, produce, want, src)
    pre, _CB._PENDING[0] = _CB._PENDING[0], None
    _CB.tag(y, key, pre)
    return y


def eligible_nhwc(x_nhwc, w, groups):
    """Shape / layout conditions of _ConvNHWC (the per-direction choice needs the hand-written side to exist
    for at least the forward)."""
    if not (x_nhwc.is_cuda and x_nhwc.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    if x_nhwc.dim() != 4 or w.dim() != 4 or groups != 1 or not x_nhwc.is_contiguous() or x_nhwc.numel() == 0:
        return False
    if not L.hip_enabled_for(x_nhwc):
        return False
    cin, cout = x_nhwc.shape[3], w.shape[0]
    if tuple(w.shape[2:]) == (1, 1):
        return L.has("pa_gemm_bf16") and cin % 64 == 0 and cout % 64 == 0
    return L.has("pa_conv2d_nhwc_fwd") and cin % 64 == 0 and cout % 8 == 0


def eligible_implicit(x_nhwc, w, groups):
    if not (x_nhwc.is_cuda and x_nhwc.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    if x_nhwc.dim() != 4 or w.dim() != 4 or groups != 1 or not x_nhwc.is_contiguous():
        return False
    if not L.has("pa_conv2d_nhwc_fwd") or not L.hip_enabled_for(x_nhwc):
        return False
    return x_nhwc.shape[3] % 64 == 0 and w.shape[0] % 8 == 0 and x_nhwc.numel() > 0


def conv_implicit_nhwc(x, w, b, stride, pad, dil, fallback):
    """KxK NHWC convolution: implicit-GEMM forward when it measured faster than MIOpen for this shape."""
    key = ("convKxK", tuple(x.shape), tuple(w.shape), stride, pad, dil, b is not None,
           x.requires_grad or w.requires_grad)

    def run(xx, ww):
        return _ConvImplicit.apply(xx, ww, b, stride, pad, dil)

    def bench(fn):
        def go():
            xx = x.detach().requires_grad_(x.requires_grad)
            ww = w.detach().requires_grad_(w.requires_grad)
            with torch.enable_grad():
                y = fn(xx, ww)
                if y.requires_grad:
                    y.backward(torch.ones_like(y))
        return go
    if not G.known(key) and not G._capturing() and L.flag("FLAGS_gemm_backend", "auto") == "auto":
        G.choose(key, {"hip": bench(run), "blas": bench(fallback)})
    if G.choose(key, {"hip": None, "blas": None}) == "hip":
        return run(x, w)
    return None


# ---------------------------------------------------------------------------------------------------- 3-D (NDHWC)
def _conv3d_own(x, w, b, stride, pads, dil):
    """Forward on the implicit GEMM (pa_conv3d_ndhwc_fwd): x [N, D, H, W, C], w [Cout, C, KD, KH, KW]."""
    N, D, H, W, C = x.shape
    Cout, _, KD, KH, KW = w.shape
    pd, ph, pw = pads
    Do = (D + 2 * pd - dil * (KD - 1) - 1) // stride + 1
    Ho = (H + 2 * ph - dil * (KH - 1) - 1) // stride + 1
    Wo = (W + 2 * pw - dil * (KW - 1) - 1) // stride + 1
    wk = w.permute(0, 2, 3, 4, 1).contiguous()
    out = torch.empty(N, Do, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    L.call("pa_conv3d_ndhwc_fwd", L.ptr(x), L.ptr(wk), L.ptr(b), L.ptr(out), L.ptr(_zero_page(x.device)), N, D, H, W,
           C, Cout, KD, KH, KW, stride, pd, ph, pw, dil, Do, Ho, Wo, L.stream_ptr())
    return out


def _conv3d_mi(x, w, b, stride, pads, dil):
    y = torch.nn.functional.conv3d(x.permute(0, 4, 1, 2, 3), w, b, stride, pads, dil)
    return y.permute(0, 2, 3, 4, 1).contiguous()


class _Conv3dNDHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pads, dil):
        key = ("conv3f", tuple(x.shape), tuple(w.shape), stride, pads, dil, b is not None)
        ch = _pick(key, lambda: _conv3d_own(x, w, b, stride, pads, dil), lambda: _conv3d_mi(x, w, b, stride, pads, dil))
        y = _conv3d_own(x, w, b, stride, pads, dil) if ch == "hip" else _conv3d_mi(x, w, b, stride, pads, dil)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pads, dil, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pads, dil, has_b = ctx.cfg
        dy = dy.contiguous()
        mask = [ctx.needs_input_grad[0], ctx.needs_input_grad[1], has_b and ctx.needs_input_grad[2]]
        gi = None
        if mask[0] and _dgrad3d_own_ok(x, w, stride, pads, dil):
            key = ("conv3d", tuple(x.shape), tuple(w.shape), stride, pads, dil)
            ch = _pick(key, lambda: _dgrad3d_own(dy, w, pads, dil), lambda: _dgrad3d_mi(dy, x, w, stride, pads, dil))
            gi = _dgrad3d_own(dy, w, pads, dil) if ch == "hip" else _dgrad3d_mi(dy, x, w, stride, pads, dil)
            mask[0] = False
        gi2, gw, gb = torch.ops.aten.convolution_backward(
            dy.permute(0, 4, 1, 2, 3), x.permute(0, 4, 1, 2, 3), w, [w.shape[0]] if has_b else None, [stride] * 3,
            list(pads), [dil] * 3, False, [0, 0, 0], 1, mask) if any(mask) else (None, None, None)
        if gi2 is not None:
            gi = gi2.permute(0, 2, 3, 4, 1).contiguous()
        return gi, gw, gb, None, None, None


def _dgrad3d_own_ok(x, w, stride, pads, dil):
    """Stride-1 data gradient as a forward convolution of dY (Cout channels in) on the implicit GEMM: the kernel's
    input-channel tile needs Cout % 64, its output C % 8, and the mirrored padding dil (K - 1) - p >= 0."""
    if stride != 1 or not L.has("pa_conv3d_ndhwc_fwd") or w.shape[0] % 64 or x.shape[4] % 8:
        return False
    return all(dil * (k - 1) - p >= 0 for k, p in zip(w.shape[2:], pads))


def _dgrad3d_own(dy, w, pads, dil):
    """dX = conv3d(dY, W flipped in every tap dim with in / out channels swapped, padding dil (K - 1) - p), NDHWC."""
    wf = w.flip(2, 3, 4).transpose(0, 1)  # [C, Cout, KD, KH, KW]
    pd = tuple(dil * (k - 1) - p for k, p in zip(w.shape[2:], pads))
    return _conv3d_own(dy, wf, None, 1, pd, dil)


def _dgrad3d_mi(dy, x, w, stride, pads, dil):
    gi = torch.ops.aten.convolution_backward(
        dy.permute(0, 4, 1, 2, 3), x.permute(0, 4, 1, 2, 3), w, None, [stride] * 3, list(pads), [dil] * 3, False,
        [0, 0, 0], 1, [True, False, False])[0]
    return gi.permute(0, 2, 3, 4, 1).contiguous()


def conv3d_ndhwc_ok(x, w, groups, stride, pads, dil):
    """Conditions of the 3-D implicit GEMM forward: bf16 NDHWC, groups 1, C % 64, Cout % 8, cubic stride."""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 5 and groups == 1):
        return False
    if not x.is_contiguous() or not L.hip_enabled_for(x) or not L.has("pa_conv3d_ndhwc_fwd"):
        return False
    return x.shape[4] % 64 == 0 and w.shape[0] % 8 == 0 and x.numel() < (1 << 31)


def conv3d_ndhwc(x, w, b, stride, pads, dil):
    """NDHWC 3-D convolution: forward, and the stride-1 data gradient (a forward convolution of dY with the flipped,
    in/out-swapped filter), each on the faster of the hand-written implicit GEMM and MIOpen (timed per shape); the
    weight gradient on MIOpen."""
    return _Conv3dNDHWC.apply(x, w, b, int(stride), tuple(int(p) for p in pads), int(dil))
