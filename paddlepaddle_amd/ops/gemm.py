"""Hand-written CDNA4 bf16 GEMM (csrc/kernels/gemm.hip) with fused epilogues.

Reference: paddle/phi/kernels/gpu/matmul_kernel.cu, paddle/phi/kernels/fusion/gpu/fused_gemm_epilogue_kernel.cu.

``gemm(a, b)`` takes 2-D views of any row/column-major layout (a transposed view is read in place — the
kernel has K-major and MN-major operand paths, so ``x.t() @ dy`` needs no copy) and fuses
``+ bias``, tanh-GELU (optionally storing the pre-activation), ``alpha`` scaling and in-place accumulation
into an existing output (fp32 or bf16) into the GEMM epilogue.
"""
from __future__ import annotations

import json
import os

import torch

from . import _loader as L

EPI_BIAS, EPI_GELU, EPI_AUX, EPI_ACCUM, EPI_OUT_F32 = 1, 2, 4, 8, 16


def _layout(t, outer_dim):
    """(ld, kmajor) of a 2-D operand whose K dimension is ``1 - outer_dim``; None if unsupported."""
    s0, s1 = t.stride()
    kdim = 1 - outer_dim
    if t.stride(kdim) == 1 and t.shape[kdim] >= 1:
        ld = t.stride(outer_dim)
        return (ld if t.shape[outer_dim] > 1 else t.shape[kdim]), True
    if t.stride(outer_dim) == 1:
        ld = t.stride(kdim)
        return (ld if t.shape[kdim] > 1 else t.shape[outer_dim]), False
    return None


def supported(a, b, out_dtype=None):
    """Shape/layout/dtype conditions of the HIP kernel for C = a @ b."""
    if a.dim() != 2 or b.dim() != 2 or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        return False
    if not L.has("pa_gemm_bf16") or not L.hip_enabled_for(a):
        return False
    M, K = a.shape
    N = b.shape[1]
    if K % 64 or N % 8 or K == 0:
        return False
    la, lb = _layout(a, 0), _layout(b, 1)
    if la is None or lb is None or la[0] % 8 or lb[0] % 8:
        return False
    if not la[1] and M % 8:
        return False
    if a.data_ptr() % 16 or b.data_ptr() % 16:
        return False
    return True


def gemm(a, b, bias=None, gelu=False, aux=None, out=None, accumulate=False, alpha=1.0, out_dtype=None, bn=None):
    """C = epi(alpha * a @ b). ``aux`` (bf16 [M, N]) receives the pre-activation when ``gelu``;
    ``accumulate`` adds into ``out`` (bf16 or fp32, [M, N] contiguous rows)."""
    M, K = a.shape
    N = b.shape[1]
    lda, ak = _layout(a, 0)
    ldb, bk = _layout(b, 1)
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype or torch.bfloat16, device=a.device)
    assert out.stride(1) == 1 and out.stride(0) % 4 == 0
    flags = 0
    if bias is not None:
        flags |= EPI_BIAS
    if gelu:
        flags |= EPI_GELU
    if aux is not None:
        flags |= EPI_AUX
        assert aux.stride(0) == out.stride(0) and aux.dtype == torch.bfloat16
    if accumulate:
        flags |= EPI_ACCUM
    if out.dtype == torch.float32:
        flags |= EPI_OUT_F32
    if bn is None:
        bn = _pick_bn(M, N, bk)
    if bn in (1, 2) and L.has("pa_gemm_bf16_pp"):
        # 256x256 + balanced tail: 1 8-wave ping-pong, 2 4-wave K32 ring
        nb = int(L.lib().pa_gemm_pp_ws_bytes(M, N, K))
        ws = torch.empty(nb // 4, dtype=torch.float32, device=a.device) if nb else None
        fn = {1: "pa_gemm_bf16_pp", 2: "pa_gemm_bf16_4w"}[bn]
        L.call(fn, L.ptr(a), L.ptr(b), L.ptr(out), L.ptr(bias),
               L.ptr(aux), M, N, K, lda, ldb, out.stride(0), int(ak), int(bk), flags, float(alpha), L.ptr(ws),
               L.stream_ptr())
        return out
    L.call("pa_gemm_bf16", L.ptr(a), L.ptr(b), L.ptr(out), L.ptr(bias), L.ptr(aux), M, N, K, lda, ldb, out.stride(0),
           int(ak), int(bk), flags, float(alpha), int(bn), 1, L.stream_ptr())
    return out


def res_supported(a, b, res):
    """pa_gemm_bf16_res conditions: the ping-pong kernel takes a @ b, residual [M, N] bf16 contiguous rows."""
    return (supported(a, b) and L.has("pa_gemm_bf16_res") and res.dtype == torch.bfloat16 and res.dim() == 2
            and tuple(res.shape) == (a.shape[0], b.shape[1]) and res.stride(1) == 1
            and res.stride(0) == b.shape[1] and res.data_ptr() % 16 == 0 and b.shape[1] % 8 == 0)


def gemm_res(a, b, res, bias=None):
    """a @ b (+ bias) + res in one launch (csrc/kernels/gemm.hip pa_gemm_bf16_res: the residual is read by the
    epilogue), ping-pong kernel with its balanced tail."""
    M, K = a.shape
    N = b.shape[1]
    lda, ak = _layout(a, 0)
    ldb, bk = _layout(b, 1)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    nb = int(L.lib().pa_gemm_pp_ws_bytes(M, N, K))
    ws = torch.empty(nb // 4, dtype=torch.float32, device=a.device) if nb else None
    L.call("pa_gemm_bf16_res", L.ptr(a), L.ptr(b), L.ptr(out), L.ptr(bias), L.ptr(res), M, N, K, lda, ldb, N,
           int(ak), int(bk), L.ptr(ws), L.stream_ptr())
    return out


def gemm_dgelu_supported(a, b, pre):
    """pa_gemm_bf16_dgelu conditions: a bf16 GEMM the 256x256 kernels take, pre-activation [M, N] bf16 rows."""
    return (supported(a, b) and L.has("pa_gemm_bf16_dgelu") and pre.dtype == torch.bfloat16 and pre.dim() == 2
            and tuple(pre.shape) == (a.shape[0], b.shape[1]) and pre.stride(1) == 1 and pre.stride(0) == b.shape[1]
            and pre.data_ptr() % 16 == 0 and b.shape[1] % 8 == 0)


def gemm_dgelu(a, b, pre, kern=1):
    """(dh, parts): dh = (a @ b) * gelu_tanh'(pre) (bf16) and the per-256-row-tile column sums of dh
    (fp32 [ceil(M / 256), N]; fold with pa_fold_partials for the bias gradient). kern: 1 ping-pong, 2 4-wave K32
    (csrc/kernels/gemm.hip pa_gemm_bf16_dgelu)."""
    M, K = a.shape
    N = b.shape[1]
    lda, ak = _layout(a, 0)
    ldb, bk = _layout(b, 1)
    dh = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    parts = torch.empty(-(-M // 256), N, dtype=torch.float32, device=a.device)
    L.call("pa_gemm_bf16_dgelu", L.ptr(a), L.ptr(b), L.ptr(dh), L.ptr(pre), L.ptr(parts), M, N, K, lda, ldb, N,
           int(ak), int(bk), int(kern), L.stream_ptr())
    return dh, parts


def _seg_table(rows):
    return torch.tensor(rows, dtype=torch.int64)  # host [nseg][5]: a_ptr, b_ptr, lda, ldb, end


def gemm_kseg_supported(As, Bs):
    """C = sum_i As[i] @ Bs[i] as one K-segmented launch: 1-4 segments, every pair passes ``supported``, the same
    operand layouts in every segment, each K_i % 64 == 0, equal M / N."""
    if not (L.has("pa_gemm_bf16_pp_segs") and 1 <= len(As) <= 4 and len(As) == len(Bs)):
        return False
    M, N = As[0].shape[0], Bs[0].shape[1]
    la, lb = None, None
    for a, b in zip(As, Bs):
        if a.shape[0] != M or b.shape[1] != N or a.shape[1] != b.shape[0] or a.shape[1] % 64 or not supported(a, b):
            return False
        ka, kb = _layout(a, 0)[1], _layout(b, 1)[1]
        if la is None:
            la, lb = ka, kb
        elif (ka, kb) != (la, lb):
            return False
    return True


def gemm_kseg(As, Bs, out=None, accumulate=False, alpha=1.0):
    """C = alpha * sum_i As[i] @ Bs[i] (``accumulate``: C +=) as ONE GEMM over K = sum K_i whose K-tiles read the
    operand pair of their segment (csrc/kernels/gemm.hip pa_gemm_bf16_pp_segs, seg_k = 1): the data gradient of
    sibling linears that share an input (dx = sum dy_i W_i^T), the weight gradients of two accumulation micro-batches
    (ops/linear.py pair_weight_grads) — one launch, one output pass, no concatenated copies."""
    M, N = As[0].shape[0], Bs[0].shape[1]
    K = sum(a.shape[1] for a in As)
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=As[0].device)
    assert out.stride(1) == 1 and out.stride(0) % 4 == 0
    rows, end = [], 0
    for a, b in zip(As, Bs):
        end += a.shape[1]
        rows.append([a.data_ptr(), b.data_ptr(), _layout(a, 0)[0], _layout(b, 1)[0], end])
    ak, bk = _layout(As[0], 0)[1], _layout(Bs[0], 1)[1]
    flags = (EPI_ACCUM if accumulate else 0) | (EPI_OUT_F32 if out.dtype == torch.float32 else 0)
    nb = int(L.lib().pa_gemm_pp_ws_bytes(M, N, K))
    ws = torch.empty(nb // 4, dtype=torch.float32, device=out.device) if nb else None
    tab = _seg_table(rows)
    rc = L.call("pa_gemm_bf16_pp_segs", tab.data_ptr(), len(rows), 1, L.ptr(As[0]), L.ptr(Bs[0]), L.ptr(out),
                L.ptr(None), M, N, K, rows[0][2], rows[0][3], out.stride(0), int(ak), int(bk), flags, float(alpha),
                L.ptr(ws), L.stream_ptr())
    if rc:
        raise RuntimeError(f"pa_gemm_bf16_pp_segs (K) failed ({rc}) for M={M} N={N} K={K}")
    return out


def gemm_nseg_supported(a, Bs):
    """C = a @ [Bs[0] | Bs[1] | ...] as one N-segmented launch: 1-4 segments of the same layout and K, every
    segment but the last 128-column aligned."""
    if not (L.has("pa_gemm_bf16_pp_segs") and 1 <= len(Bs) <= 4):
        return False
    K = a.shape[1]
    lay = None
    for i, b in enumerate(Bs):
        if b.shape[0] != K or not supported(a, b) or (i + 1 < len(Bs) and b.shape[1] % 128):
            return False
        kb = _layout(b, 1)[1]
        if lay is None:
            lay = kb
        elif kb != lay:
            return False
    return True


def gemm_nseg(a, Bs, out=None, alpha=1.0):
    """C [M, sum N_i] = alpha * a @ [Bs[0] | Bs[1] | ...] as ONE GEMM whose column tiles read the weight of their
    segment (pa_gemm_bf16_pp_segs, seg_k = 0): the q / k / v or gate / up projections of one input with separate
    weight tensors, no concatenated weight copy; the per-projection outputs are column views of C."""
    M, K = a.shape
    N = sum(b.shape[1] for b in Bs)
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    assert out.stride(1) == 1 and out.stride(0) % 4 == 0
    rows, end = [], 0
    for b in Bs:
        end += b.shape[1]
        rows.append([a.data_ptr(), b.data_ptr(), _layout(a, 0)[0], _layout(b, 1)[0], end])
    lda, ak = _layout(a, 0)
    bk = _layout(Bs[0], 1)[1]
    flags = EPI_OUT_F32 if out.dtype == torch.float32 else 0
    nb = int(L.lib().pa_gemm_pp_ws_bytes(M, N, K))
    ws = torch.empty(nb // 4, dtype=torch.float32, device=a.device) if nb else None
    tab = _seg_table(rows)
    rc = L.call("pa_gemm_bf16_pp_segs", tab.data_ptr(), len(rows), 0, L.ptr(a), L.ptr(Bs[0]), L.ptr(out),
                L.ptr(None), M, N, K, lda, rows[0][3], out.stride(0), int(ak), int(bk), flags, float(alpha),
                L.ptr(ws), L.stream_ptr())
    if rc:
        raise RuntimeError(f"pa_gemm_bf16_pp_segs (N) failed ({rc}) for M={M} N={N} K={K}")
    return out


def gemm_seg_supported(a1, a2, b1, b2):
    return gemm_kseg_supported([a1, a2], [b1, b2])


def gemm_seg(a1, a2, b1, b2, out=None, accumulate=False, alpha=1.0):
    """C = alpha * (a1 @ b1 + a2 @ b2): the two-segment case of ``gemm_kseg``."""
    return gemm_kseg([a1, a2], [b1, b2], out=out, accumulate=accumulate, alpha=alpha)


def gemm_bn_stats(a, b, bias=None, bn=None):
    """C = a @ b (+ bias) in bf16 plus the batch-norm partials of C's columns, written by the GEMM epilogue
    (kEpiStats): returns (C, stats [2 * chunks * N] fp32, chunks) for ops/bn.py (conv -> BN fusion).
    bn: tile width (160: three-stage kernel; 128 / 256: two-stage kernel), default by layout."""
    M, K = a.shape
    N = b.shape[1]
    lda, ak = _layout(a, 0)
    ldb, bk = _layout(b, 1)
    if bn is None:
        bn = 160 if bk else (256 if _pick_bn(M, N, bk) == 256 else 128)
    chunks = int(L.lib().pa_gemm_stats_chunks(M, bn))
    out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    stats = torch.empty(2 * chunks * N, dtype=torch.float32, device=a.device)
    L.call("pa_gemm_bf16_stats", L.ptr(a), L.ptr(b), L.ptr(out), L.ptr(bias), M, N, K, lda, ldb, N, int(ak),
           int(bk), EPI_BIAS if bias is not None else 0, bn, L.ptr(stats), L.stream_ptr())
    return out, stats, chunks


def gemm_splitk(a, b, splits, out_dtype=torch.bfloat16, bn=None):
    """C = a @ b with K split over ``splits`` slices computed by separate workgroups (fp32 slabs, summed
    here): fills the chip when M x N has few tiles but K is long (weight gradients of convolutions)."""
    M, K = a.shape
    N = b.shape[1]
    lda, ak = _layout(a, 0)
    ldb, bk = _layout(b, 1)
    ws = torch.empty(splits, M, N, dtype=torch.float32, device=a.device)
    if bn is None:
        bn = _pick_bn(M, N, bk)
    L.call("pa_gemm_bf16", L.ptr(a), L.ptr(b), L.ptr(ws), L.ptr(None), L.ptr(None), M, N, K, lda, ldb, N,
           int(ak), int(bk), EPI_OUT_F32, 1.0, int(bn), int(splits), L.stream_ptr())
    return reduce_slabs(ws, out_dtype)


def pp_splits(M, N, K, cus=256, max_ws_bytes=256 << 20):
    """K-split factor of the ping-pong split-K GEMM: 1-2 workgroups per CU, slices of >= 4 K-tiles (64), fp32
    partial tiles within the workspace budget; 0 when no split fits."""
    T = -(-M // 256) * -(-N // 256)
    nk = K // 64
    s = 1
    while T * s * 2 <= 2 * cus and nk % (s * 2) == 0 and nk // (s * 2) >= 4 and T * s * 2 * 262144 <= max_ws_bytes:
        s *= 2
    return s if s > 1 else 0


def gemm_pp_splitk_ok(a, b, splits):
    if not (splits and L.has("pa_gemm_bf16_pp_splitk") and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and a.is_cuda and L.hip_enabled_for(a)):
        return False
    M, K = a.shape
    N = b.shape[1]
    la, lb = _layout(a, 0), _layout(b, 1)
    return (la is not None and lb is not None and K % 64 == 0 and (K // 64) % splits == 0 and N % 8 == 0
            and la[0] % 8 == 0 and lb[0] % 8 == 0 and (la[1] or M % 8 == 0))


def gemm_pp_splitk(a, b, splits, out_dtype=torch.bfloat16, out=None, accumulate=False):
    """C = a @ b on the ping-pong 256x256 kernel with every tile cut into ``splits`` K slices (fp32 partial tiles
    summed, with the cast, by the tail-reduction kernel): the split-K form for few output tiles and a long K.
    ``out`` + ``accumulate``: C += a @ b in place (the reduction reads C; gradient-accumulation fusion)."""
    M, K = a.shape
    N = b.shape[1]
    lda, ak = _layout(a, 0)
    ldb, bk = _layout(b, 1)
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=a.device)
    elif out.shape != (M, N) or out.stride(1) != 1 or out.stride(0) % 4 or out.dtype not in (torch.bfloat16,
                                                                                           torch.float32):
        raise ValueError("gemm_pp_splitk: out must be a row-major [M, N] bf16 / fp32 tensor")
    ws = torch.empty(int(L.lib().pa_gemm_pp_splitk_ws_bytes(M, N, splits)) // 4, dtype=torch.float32,
                     device=a.device)
    flags = (EPI_OUT_F32 if out.dtype == torch.float32 else 0) | (EPI_ACCUM if accumulate else 0)
    L.call("pa_gemm_bf16_pp_splitk", L.ptr(a), L.ptr(b), L.ptr(out), M, N, K, lda, ldb, out.stride(0), int(ak),
           int(bk), flags, 1.0, int(splits), L.ptr(ws), L.stream_ptr())
    return out


def reduce_slabs(ws, out_dtype):
    """[splits, M, N] fp32 split-K partials -> [M, N] out_dtype; bf16 in one HIP pass (sum + cast)."""
    splits, M, N = ws.shape
    if out_dtype == torch.bfloat16 and N % 4 == 0 and L.has("pa_slab_reduce_bf16"):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=ws.device)
        L.call("pa_slab_reduce_bf16", L.ptr(ws), L.ptr(out), N, M, N, int(splits), L.stream_ptr())
        return out
    return ws.sum(0, dtype=torch.float32).to(out_dtype) if splits > 1 else ws[0].to(out_dtype)


def skinny_supported(a, b):
    """gemm_skinny's conditions: bf16, A row-major, tall M, N and K in {32, 64, 128, 256}, 16-byte rows."""
    if not (L.has("pa_gemm_skinny") and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.is_cuda):
        return False
    M, K = a.shape
    N = b.shape[1]
    if a.stride(1) != 1 or a.stride(0) % 8 or M < 1024 or not L.lib().pa_gemm_skinny_ok(N, K):
        return False
    return (b.stride(0) == 1 and b.stride(1) % 8 == 0) or (b.stride(1) == 1 and b.stride(0) % 8 == 0)


def gemm_skinny(a, b, bias=None, out=None, accumulate=False, relu=False):
    """C = a @ b (+ bias) (relu), or C += a @ b with ``accumulate``: the memory-bound kernel for a tall M and a
    small N x K (csrc/kernels/gemm_skinny.hip; the 1x1 convolutions of ResNet's early stages)."""
    M, K = a.shape
    N = b.shape[1]
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    assert out.stride(1) == 1 and out.stride(0) % 8 == 0 and out.dtype == torch.bfloat16
    bk = b.stride(0) == 1  # b = B^T row-major viewed transposed
    ldb = b.stride(1) if bk else b.stride(0)
    flags = (1 if bias is not None else 0) | (2 if accumulate else 0) | (4 if relu else 0)
    rc = L.call("pa_gemm_skinny", L.ptr(a), L.ptr(b), L.ptr(out), L.ptr(bias), M, N, K, a.stride(0), ldb,
                out.stride(0), int(bk), flags, L.stream_ptr())
    if rc:
        raise RuntimeError(f"pa_gemm_skinny failed ({rc}) for M={M} N={N} K={K}")
    return out


def gemm_skinny_bn_stats(a, b, bias=None):
    """gemm_skinny plus the batch-norm partials of C's columns (N <= 128): (C, stats, chunks), or None when the
    shape has no statistics variant."""
    M, K = a.shape
    N = b.shape[1]
    chunks = int(L.lib().pa_gemm_skinny_stats_chunks(M, N, K))
    if chunks <= 0:
        return None
    out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    stats = torch.empty(2 * chunks * N, dtype=torch.float32, device=a.device)
    bk = b.stride(0) == 1
    ldb = b.stride(1) if bk else b.stride(0)
    L.call("pa_gemm_skinny_stats", L.ptr(a), L.ptr(b), L.ptr(out), L.ptr(bias), M, N, K, a.stride(0), ldb, N, int(bk),
           L.ptr(stats), L.stream_ptr())
    return out, stats, chunks


def pick_splits(M, N, K, bn=256, cus=256, max_ws_bytes=256 << 20):
    """Largest power-of-two split keeping K-slices a multiple of 64 that brings the grid to ~2 waves."""
    tiles = -(-M // 256) * -(-N // bn)
    s = 1
    while tiles * s * 2 <= 2 * cus and K % (s * 2 * 64) == 0 and (s * 2) * M * N * 4 <= max_ws_bytes:
        s *= 2
    return s


def _pick_bn(M, N, b_kmajor, cus=256):
    """Kernel variant. Measured on MI355X (profiles/gemm_mfma_vs_hipblaslt.log): the 4-phase ping-pong
    256x256 kernel (code 1, with the balanced K-split tail) is the fastest of ours on every layout once the
    output fills a wave of 256x256 tiles with M, N >= 1024. Below that: the 3-stage 256x160 kernel
    whenever B is K-major (its 160-column MN-major image would read unaligned 320-B rows); otherwise the
    2-stage 256x256 kernel, or 256x128 when that fills the CUs better."""
    if M >= 1024 and N >= 1024 and -(-M // 256) * -(-N // 256) >= cus:
        return 1
    if b_kmajor:
        return 160

    def eff(bn):
        t = -(-M // 256) * -(-N // bn)
        waves = -(-t // cus)
        return t / (waves * cus) * (1.0 if bn == 256 else 0.9)
    return 256 if eff(256) >= eff(128) else 128


# ---------------------------------------------------------------------------------------------
# Per-shape backend choice. For every (product, shape, layout, epilogue) key the first eager call
# times the hand-written kernel (fused epilogue) against hipBLASLt (+ the separate epilogue pass)
# on scratch outputs and keeps the faster one — our own TunableOp. Inside a hipGraph capture no
# timing happens (hipBLASLt is used until the key has been tuned eagerly).
# FLAGS_gemm_backend = "auto" (default) | "hip" | "blas" forces a side.
#
# Decisions persist: paddlepaddle_amd/ops/tuning/<arch>.json (committed, measured on MI355X) is read first,
# so every process makes the same choice for a known shape without timing it (and a captured graph uses the
# tuned kernel); shapes it does not hold are timed once and appended to the per-user overlay
# $PADDLE_AMD_TUNING_FILE (default ~/.cache/paddlepaddle_amd/tuning_<arch>.json), read on later starts.
_CHOICE = {}
_TABLE_LOADED = False
_TUNING_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning")


def _arch():
    try:
        return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]
    except Exception:  # pragma: no cover
        return "unknown"


def _canon(key):
    """Decision keys as JSON-stable tuples (dtypes and other objects by their str; nested tuples flattened
    to lists and back)."""
    def c(v):
        if isinstance(v, (bool, int, float, str)) or v is None:
            return v
        if isinstance(v, (tuple, list)):
            return tuple(c(x) for x in v)
        return str(v)
    return tuple(c(v) for v in key)


def _key_str(key):
    def j(v):
        return [j(x) for x in v] if isinstance(v, tuple) else v
    return json.dumps([j(v) for v in key])


def known(key):
    """Whether a decision for ``key`` exists (committed table, overlay or measured in this process)."""
    load_tuning_table()
    return _canon(key) in _CHOICE


# bumped whenever what "hip" runs for a key changes (v2: the ping-pong kernel for large GEMMs), so
# decisions timed against an older kernel set are not reused
_TABLE_VERSION = 2


def _overlay_path():
    return os.environ.get("PADDLE_AMD_TUNING_FILE") or os.path.join(
        os.path.expanduser("~"), ".cache", "paddlepaddle_amd", f"tuning_{_arch()}_v{_TABLE_VERSION}.json")


def _read_table(path):
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("version", 1) != _TABLE_VERSION:
            return {}
        return {_canon(json.loads(k)): v for k, v in d.get("choices", {}).items()}
    except (OSError, ValueError):
        return {}


def load_tuning_table():
    """Merge the committed table and the overlay into the in-process decisions (once per process)."""
    global _TABLE_LOADED
    if _TABLE_LOADED:
        return
    _TABLE_LOADED = True
    if os.environ.get("PADDLE_AMD_TUNING_RETUNE", "0") == "1":  # re-time every key (table refresh runs)
        return
    for path in (os.path.join(_TUNING_DIR, f"{_arch()}.json"), _overlay_path()):
        for k, v in _read_table(path).items():
            _CHOICE.setdefault(k, v)


def _persist(key, choice):
    path = _overlay_path()
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        cur = {}
        if os.path.exists(path):
            with open(path) as f:
                cur = json.load(f).get("choices", {})
        cur[_key_str(key)] = choice
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump({"arch": _arch(), "version": _TABLE_VERSION, "choices": cur}, f, indent=0, sort_keys=True)
        os.replace(tmp, path)
    except OSError:  # read-only home: the decision still holds for this process
        pass


def dump_tuning_table(path):
    """Write every decision of this process (committed-table format)."""
    with open(path, "w") as f:
        json.dump({"arch": _arch(), "version": _TABLE_VERSION,
                   "choices": {_key_str(k): v for k, v in sorted(_CHOICE.items(), key=str)}}, f, indent=0,
                  sort_keys=True)


def _capturing():
    try:
        return torch.cuda.is_current_stream_capturing()
    except Exception:  # pragma: no cover
        return False


def _flush_caches(dev):
    """Evict L2 and the 256 MB MALL (Infinity Cache): write a 512 MB scratch buffer (skipped when the device
    has no room for it — the timing is then warm, which only biases the choice, never breaks it)."""
    try:
        buf = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    except torch.cuda.OutOfMemoryError:
        return None
    buf.zero_()
    return buf


def _spin():
    try:
        torch.cuda._sleep(2_000_000)  # ~1 ms of device spin ahead of the timed launches
    except Exception:  # pragma: no cover
        pass


def choose(key, candidates, cold=False):
    """Name of the faster entry of ``candidates`` ({name: zero-arg callable without side effects}).
    ``cold``: time every call after evicting the caches — for weight-streaming (decode) GEMMs, whose weights
    come from HBM in a real step (the whole model streams through) but would sit in the 256 MB MALL when one
    GEMM is repeated."""
    mode = L.flag("FLAGS_gemm_backend", "auto")
    if mode in candidates:
        return mode
    load_tuning_table()
    key = _canon(key)
    _USED.add(key)
    ch = _CHOICE.get(key)
    if ch is not None and ch in candidates:
        return ch
    if _capturing():
        return "blas"
    if not L.flag("FLAGS_use_autotune", True):  # incubate.autotune kernel tuning off: no timing, vendor GEMM
        return "blas" if "blas" in candidates else next(iter(candidates))
    times = {n: [] for n in candidates}
    for fn in candidates.values():
        fn()
    dev = torch.cuda.current_device()
    for _ in range(3):
        for n, fn in candidates.items():
            if cold:
                _flush_caches(dev)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # keep the GPU busy while the candidate's launches are issued, so the events bracket device time
            # only: host launch cost (ctypes / Python) would otherwise count against the hand-written side
            _spin()
            s.record()
            fn()
            e.record()
            e.synchronize()
            times[n].append(s.elapsed_time(e))
    ch = min(times, key=lambda n: min(times[n]))
    _CHOICE[key] = ch
    _persist(key, ch)
    return ch


_USED = set()


def choices(used_only=True):
    """Decisions {key: backend} (for logs / profiles): by default only the keys this process dispatched."""
    if used_only:
        return {k: v for k, v in _CHOICE.items() if k in _USED}
    return dict(_CHOICE)


# ---------------------------------------------------------------------------------------------
# Decode-shape GEMM (M <= 64 rows x a weight in paddle's [in, out] layout): bandwidth-bound on the
# weight, so the kernel streams it with a 4-deep glds ring and splits K over workgroups to fill the chip.
def small_m_supported(a, b):
    if a.dim() != 2 or b.dim() != 2 or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        return False
    if not L.has("pa_gemm_small_m") or not L.hip_enabled_for(a):
        return False
    M, K = a.shape
    N = b.shape[1]
    return (1 <= M <= 64 and a.stride(1) == 1 and a.stride(0) % 8 == 0 and b.stride(1) == 1 and b.stride(0) % 8 == 0
            and N % 8 == 0 and K % 64 == 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)


def gemm_small_m(a, b, bias=None, splits=None, cus=256, stages=4):
    M, K = a.shape
    N = b.shape[1]
    if splits is None:
        blocks = -(-N // 128)
        splits = 1
        while blocks * splits * 2 <= 2 * cus and K % (64 * splits * 2) == 0 and K // (splits * 2) >= 256:
            splits *= 2
    out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    ws = torch.empty(splits * M * N if splits > 1 else 1, dtype=torch.float32, device=a.device)
    L.call("pa_gemm_small_m", L.ptr(a), a.stride(0), L.ptr(b), b.stride(0), L.ptr(out), out.stride(0), L.ptr(bias),
           L.ptr(ws), M, N, K, int(splits), int(stages), L.stream_ptr())
    return out


def small_m_variants(M, N, K, cus=256):
    """(splits, stages) candidates for a decode GEMM, timed by the autotuner: split counts that divide the
    K tiles (at least 4 K-tiles per workgroup) and put between ~0.5 and 4 workgroups per CU, each with the
    4-stage (1 workgroup / CU) and 3-stage (2 / CU) LDS ring."""
    kt = K // 64
    blocks = -(-N // 128)
    out = []
    for d in range(1, kt + 1):
        if kt % d or kt // d < 4:
            continue
        wgs = blocks * d
        if wgs > 6 * cus or (wgs < cus // 2 and kt // d > 4 and d < kt):
            continue
        out.append(d)
    if not out:
        out = [1]
    # keep at most 4 split counts: the ones closest to 1 and 2 workgroups per CU
    out = sorted(out, key=lambda d: min(abs(blocks * d - cus), abs(blocks * d - 2 * cus)))[:4]
    return [(d, st) for d in sorted(out) for st in (4, 3)]
