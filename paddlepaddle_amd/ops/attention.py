"""Flash attention forward/backward (HIP, MFMA bf16) in paddle's [batch, seq, heads, head_dim] layout.

Reference: paddle/phi/kernels/gpu/flash_attn_kernel.cu, flash_attn_grad_kernel.cu,
python/paddle/nn/functional/flash_attention.py:364 (flash_attention), :1145 (sdpa).
Kernel: csrc/kernels/flash_attn.hip — per workgroup a 64-row (or 128-row) Q block, K/V tiles
streamed through LDS, S = QKᵀ and O += PV on v_mfma_f32_16x16x32_bf16, online softmax with the
running max/sum in registers, LSE written for the backward. GQA via kv-head = head / (H/Hk).
Backward recomputes P from Q, K and LSE (no S×S materialisation): dV, dK accumulated per key block,
dQ accumulated in fp32.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn.functional as F

from . import _loader as L
from ..framework.trace_hook import static_op


def attention_reference(q, k, v, causal=False, scale=None, mask=None, dropout=0.0, training=False, keep=None):
    """Plain math reference in fp32; q,k,v [B,S,H,D]. ``mask``: bool (True = attend) or additive, broadcastable
    to [B, H, Sq, Sk]; ``keep``: an explicit dropout keep mask [B, H, Sq, Sk] (used by the tests to replay the
    kernel's mask)."""
    B, Sq, H, D = q.shape
    Hk = k.shape[2]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    if Hk != H:
        kf = kf.repeat_interleave(H // Hk, 1)
        vf = vf.repeat_interleave(H // Hk, 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Sk = k.shape[1]
    if causal:
        cm = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        s = s.masked_fill(~cm, float("-inf"))
    if mask is not None:
        m = mask
        if m.dtype == torch.bool:
            s = s.masked_fill(~m, float("-inf"))
        else:
            s = s + m.float()
    dead = torch.isneginf(s).all(-1, keepdim=True)  # fully masked rows: zero output / gradients, as the kernel
    if bool(dead.any()):
        s = s.masked_fill(dead, 0.0)
    p = torch.softmax(s, -1)
    if bool(dead.any()):
        p = p.masked_fill(dead, 0.0)
    if keep is not None:
        p = p * keep.float() / (1.0 - dropout)
    elif dropout > 0 and training:
        p = F.dropout(p, dropout)
    o = torch.matmul(p, vf)
    return o.transpose(1, 2).to(q.dtype)


def _sdpa(q, k, v, causal, scale, mask, dropout, training):
    """ATen SDPA path: CPU, and on the GPU only for what the HIP kernel does not cover (fp32 inputs, head_dim
    > 256); counted in ops._loader.CALLS["attn_aten_fallback"] so tests can assert it did not run."""
    if q.is_cuda:
        L.CALLS["attn_aten_fallback"] = L.CALLS.get("attn_aten_fallback", 0) + 1
    qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    H, Hk = q.shape[2], k.shape[2]
    if Hk != H:
        kt = kt.repeat_interleave(H // Hk, 1)
        vt = vt.repeat_interleave(H // Hk, 1)
    am = mask
    if am is not None and am.dtype != torch.bool:
        am = am.to(q.dtype)
    if causal and q.shape[1] != k.shape[1]:
        Sq, Sk = q.shape[1], k.shape[1]
        cm = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        am = cm if am is None else (am & cm if am.dtype == torch.bool else am.masked_fill(~cm, float("-inf")))
        causal = False
    elif causal and am is not None:
        S = q.shape[1]
        cm = torch.ones(S, S, dtype=torch.bool, device=q.device).tril()
        am = am & cm if am.dtype == torch.bool else am.masked_fill(~cm, float("-inf"))
        causal = False
    o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=am, dropout_p=dropout if training else 0.0,
                                       is_causal=causal and am is None, scale=scale)
    return o.transpose(1, 2)


def _strides(t):
    st = t.stride()
    return [st[0], st[1], st[2]] if t.dim() == 4 else [0, st[0], st[1]]  # varlen [total, H, D]: no batch stride


def _i64arr(vals):
    import ctypes
    return (ctypes.c_int64 * len(vals))(*[int(v) for v in vals])


class _AttnExtra(ctypes.Structure):
    """Mirror of PaAttnExtra (csrc/kernels/flash_attn.hip): the optional terms of a launch."""
    _fields_ = [("cu_q", ctypes.c_void_p), ("cu_k", ctypes.c_void_p), ("mask", ctypes.c_void_p),
                ("mask_kind", ctypes.c_int64), ("ms", ctypes.c_int64 * 3), ("fm", ctypes.c_void_p),
                ("fm_cols", ctypes.c_int64), ("fms", ctypes.c_int64 * 2), ("fm_stats", ctypes.c_void_p),
                ("fmst", ctypes.c_int64 * 2), ("drop_p", ctypes.c_double),
                ("seed", ctypes.c_uint64), ("lse_s", ctypes.c_int64 * 2), ("dtype", ctypes.c_int64)]


_MASK_KIND = {torch.bool: 1, torch.bfloat16: 2, torch.float32: 3}


def _prep_mask(mask, B, H, Sq, Sk):
    """Mask broadcastable to [B, H, Sq, Sk] -> (tensor, kind, strides(b, h, q)) in the layout the kernel reads:
    keys contiguous, 16-byte aligned rows of a multiple of 8 keys (else a padded copy); broadcast dims stride 0."""
    m = mask
    while m.dim() < 4:
        m = m.unsqueeze(0)
    if m.dim() != 4:
        raise ValueError(f"attention mask must be broadcastable to [B, H, Sq, Sk], got {list(mask.shape)}")
    for got, want in zip(m.shape, (B, H, Sq, Sk)):
        if got not in (1, want):
            raise ValueError(f"attention mask {list(mask.shape)} does not broadcast to {[B, H, Sq, Sk]}")
    if m.dtype not in _MASK_KIND:
        m = m.to(torch.float32)
    es = m.element_size()
    ok = (m.shape[-1] == Sk and m.stride(-1) == 1 and Sk % 8 == 0 and m.data_ptr() % 16 == 0
          and (m.shape[-2] == 1 or m.stride(-2) % 8 == 0))
    if not ok:
        skp = -(-Sk // 8) * 8
        buf = torch.zeros(m.shape[0], m.shape[1], m.shape[2], skp, dtype=m.dtype, device=m.device)
        buf[..., :Sk] = m.expand(m.shape[0], m.shape[1], m.shape[2], Sk)
        m = buf
    st = [0 if m.shape[i] == 1 else m.stride(i) for i in range(3)]
    del es
    return m, _MASK_KIND[m.dtype], st


def _prep_flashmask(se, B, H, Sk):
    """startend_row_indices [B, H|1, Sk, 1|2|4] -> int32, contiguous, key dim padded to a multiple of 4."""
    t = se.to(torch.int32)
    if t.dim() != 4 or t.shape[-1] not in (1, 2, 4) or t.shape[2] != Sk:
        raise ValueError(f"startend_row_indices must be [B, H|1, Sk, 1|2|4], got {list(se.shape)}")
    skp = -(-Sk // 4) * 4
    if skp != Sk:
        t = torch.cat([t, t[:, :, :1].expand(t.shape[0], t.shape[1], skp - Sk, t.shape[3])], 2)
    t = t.contiguous()
    return t, t.shape[-1], [0 if t.shape[0] == 1 else t.stride(0), 0 if t.shape[1] == 1 else t.stride(1)]


def _draw_seed():
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


class _Job:
    """Everything one forward/backward pair of launches needs (shapes, optional terms, their tensors kept alive)."""

    def __init__(self, q, k, varlen, causal, scale, mask, startend, dropout, seed, cu_q, cu_k, max_q, max_k):
        self.varlen = varlen
        if varlen:
            self.B = cu_q.numel() - 1
            self.Sq, self.Sk = int(max_q), int(max_k)
            self.H, self.Hk, self.D = q.shape[1], k.shape[1], q.shape[2]
            self.q_rows = q.shape[0]
        else:
            self.B, self.Sq, self.H, self.D = q.shape
            self.Sk, self.Hk = k.shape[1], k.shape[2]
            self.q_rows = self.B * self.Sq
        self.causal, self.scale = bool(causal), float(scale)
        self.keep = []  # tensors referenced by pointer
        ex = _AttnExtra()
        if varlen:
            self.cu_q, self.cu_k = cu_q.to(torch.int32).contiguous(), cu_k.to(torch.int32).contiguous()
            ex.cu_q, ex.cu_k = self.cu_q.data_ptr(), self.cu_k.data_ptr()
            ex.lse_s[0], ex.lse_s[1] = 0, self.q_rows
        if mask is not None:
            m, kind, st = _prep_mask(mask, self.B, self.H, self.Sq, self.Sk)
            self.keep.append(m)
            ex.mask, ex.mask_kind = m.data_ptr(), kind
            ex.ms[0], ex.ms[1], ex.ms[2] = st
        if startend is not None:
            t, cols, st = _prep_flashmask(startend, self.B, self.H, self.Sk)
            self.keep.append(t)
            ex.fm, ex.fm_cols = t.data_ptr(), cols
            ex.fms[0], ex.fms[1] = st
            # per-64-key-tile extrema of the bounds: lets the kernels skip fully masked blocks
            Bm, Hm = t.shape[0], t.shape[1]
            nt = -(-self.Sk // 64)
            nt += nt % 2
            stats = torch.empty(Bm * Hm * nt * 8, dtype=torch.int32, device=t.device)
            L.call("pa_fa_fm_stats", L.ptr(t), int(cols), int(self.causal), int(self.Sk), int(Bm), int(Hm),
                   int(t.stride(0)), int(t.stride(1)), int(nt), L.ptr(stats), L.stream_ptr())
            self.keep.append(stats)
            ex.fm_stats = stats.data_ptr()
            ex.fmst[0], ex.fmst[1] = (0 if Bm == 1 else Hm * nt * 8), (0 if Hm == 1 else nt * 8)
        if dropout > 0:
            ex.drop_p, ex.seed = float(dropout), int(seed)
        ex.dtype = 1 if q.dtype == torch.float16 else 0
        self.ex = ex

    def lse_shape(self):
        return (self.H, self.q_rows) if self.varlen else (self.B, self.H, self.Sq)


def _fa_fwd(q, k, v, job):
    o = torch.empty_like(q) if job.varlen else torch.empty(job.B, job.Sq, job.H, job.D, dtype=q.dtype, device=q.device)
    lse = torch.empty(job.lse_shape(), dtype=torch.float32, device=q.device)
    st = _i64arr(_strides(q) + _strides(k) + _strides(v) + _strides(o))
    L.call("pa_flash_attn_fwd_ex", L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(o), L.ptr(lse), st, job.B, job.Sq, job.Sk,
           job.H, job.Hk, job.D, job.scale, int(job.causal), ctypes.addressof(job.ex), L.stream_ptr())
    return o, lse


def _ds_budget_bytes():
    import os
    return int(float(os.environ.get("PA_FA_BWD_DS_MAX_GB", "16")) * (1 << 30))


def _fa_bwd(q, k, v, o, lse, do, dq, dk, dv, job):
    delta = torch.empty(job.lse_shape(), dtype=torch.float32, device=q.device)
    st = _i64arr(_strides(q) + _strides(k) + _strides(v) + _strides(o) + _strides(do) + _strides(dq)
                 + _strides(dk) + _strides(dv))
    ex = job.ex
    lib = L.lib()
    if lib.pa_flash_attn_bwd_ds_ok(int(job.D), int(bool(ex.mask)), int(bool(ex.fm)), int(ex.drop_p > 0),
                                   int(job.varlen)):
        nbytes = int(lib.pa_flash_attn_bwd_ds_bytes(job.B, job.Sq, job.Sk, job.H))
        if nbytes <= _ds_budget_bytes():
            # dS route: unscaled dS^T tiles (16-bit) in a transient scratch, dQ = scale * dS K by its own kernel;
            # no fp32 dQ buffer / atomics / convert pass (csrc/kernels/flash_attn_kernels.h fa_bwd_dq_kernel)
            ds = torch.empty(nbytes // 2, dtype=q.dtype, device=q.device)
            L.CALLS["flash_attn_bwd_ds"] = L.CALLS.get("flash_attn_bwd_ds", 0) + 1
            L.call("pa_flash_attn_bwd_ds", L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(o), L.ptr(do), L.ptr(lse), L.ptr(dq),
                   L.ptr(dk), L.ptr(dv), L.ptr(ds), L.ptr(delta), st, job.B, job.Sq, job.Sk, job.H, job.Hk, job.D,
                   job.scale, int(job.causal), ctypes.addressof(job.ex), L.stream_ptr())
            return
    dq_acc = torch.empty(job.q_rows, job.H, job.D, dtype=torch.float32, device=q.device)
    L.call("pa_flash_attn_bwd_ex", L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(o), L.ptr(do), L.ptr(lse), L.ptr(dq),
           L.ptr(dk), L.ptr(dv), L.ptr(dq_acc), L.ptr(delta), st, job.B, job.Sq, job.Sk, job.H, job.Hk, job.D,
           job.scale, int(job.causal), int(job.q_rows), ctypes.addressof(job.ex), L.stream_ptr())


def _lastdim_contig(t):
    return t.stride(-1) == 1 and t.data_ptr() % 16 == 0 and all(s % 8 == 0 for s in t.stride()[:-1])


class _FlashAttnHIP(torch.autograd.Function):
    """q [B,Sq,H,D] / k, v [B,Sk,Hk,D] (or varlen [total, H, D] with cu_seqlens) -> (o, lse). dK / dV come out per
    KV head (the kernel sums the query heads of a group)."""

    @staticmethod
    def forward(ctx, q, k, v, job):
        q, k, v = [t if _lastdim_contig(t) else t.contiguous() for t in (q, k, v)]
        o, lse = _fa_fwd(q, k, v, job)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.job = job
        ctx.mark_non_differentiable(lse)
        return o, lse

    @staticmethod
    def backward(ctx, do, _dlse):
        q, k, v, o, lse = ctx.saved_tensors
        do = do.to(q.dtype)
        if not _lastdim_contig(do):
            do = do.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _fa_bwd(q, k, v, o, lse, do, dq, dk, dv, ctx.job)
        return dq, dk, dv, None


class _FlashAttnQKVPackedHIP(torch.autograd.Function):
    """qkv [B, S, H, 3, D] (PaddleNLP fused-QKV layout) -> o [B, S, H, D]; grad is one dqkv buffer."""

    @staticmethod
    def forward(ctx, qkv, causal, scale):
        q, k, v = qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2]
        job = _Job(q, k, False, causal, scale, None, None, 0.0, 0, None, None, None, None)
        o, lse = _fa_fwd(q, k, v, job)
        ctx.save_for_backward(qkv, o, lse)
        ctx.job = job
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        do = do.to(qkv.dtype)
        if not _lastdim_contig(do):
            do = do.contiguous()
        dqkv = torch.empty_like(qkv)
        q, k, v = qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2]
        _fa_bwd(q, k, v, o, lse, do, dqkv[:, :, :, 0], dqkv[:, :, :, 1], dqkv[:, :, :, 2], ctx.job)
        return dqkv, None, None


class _QKVRopeAttnHIP(torch.autograd.Function):
    """Fused QKV projection output t [B, S, (H + 2*Hkv) * D] (per-token layout [q heads | k heads | v heads]) ->
    RoPE(q), RoPE(k) -> causal flash attention -> o [B, S, H, D].

    Forward: one row-strided RoPE launch rotates q|k out of t into a packed [B, S, H + Hkv, D] buffer; v is read
    in place from t. Backward: the attention kernel writes dq, dk and dv straight into their column ranges of ONE
    [B, S, W] gradient buffer and one in-place inverse rotation finishes dq|dk — the unfused path's per-tensor
    rope launches, split-backward concatenation (CatArrayBatchedCopy) and its extra [B, S, W] round trip are gone.
    Reference behaviour: the q/k/v split + fused_rotary_position_embedding + flash_attention sequence of
    PaddleNLP's LlamaAttention (python/paddle/incubate/nn/functional/fused_rotary_position_embedding.py:22)."""

    @staticmethod
    def forward(ctx, t, cos, sin, H, Hkv, D, causal, scale, neox):
        B, S, W = t.shape
        if not t.is_contiguous():
            t = t.contiguous()
        qk = torch.empty(B, S, H + Hkv, D, dtype=t.dtype, device=t.device)
        L.call("pa_rope_rows", L.ptr(t), W, L.ptr(cos), L.ptr(sin), L.ptr(qk), (H + Hkv) * D, B * S, S, H + Hkv, D,
               int(neox), L.dcode(t), L.stream_ptr())
        q, k = qk[:, :, :H], qk[:, :, H:]
        v = t.view(B, S, H + 2 * Hkv, D)[:, :, H + Hkv:]
        job = _Job(q, k, False, causal, scale, None, None, 0.0, 0, None, None, None, None)
        o, lse = _fa_fwd(q, k, v, job)
        ctx.save_for_backward(t, qk, cos, sin, o, lse)
        ctx.job, ctx.dims, ctx.neox = job, (H, Hkv, D), neox
        return o

    @staticmethod
    def backward(ctx, do):
        t, qk, cos, sin, o, lse = ctx.saved_tensors
        H, Hkv, D = ctx.dims
        B, S, W = t.shape
        do = do.to(t.dtype)
        if not _lastdim_contig(do):
            do = do.contiguous()
        g = torch.empty_like(t)
        g4 = g.view(B, S, H + 2 * Hkv, D)
        v = t.view(B, S, H + 2 * Hkv, D)[:, :, H + Hkv:]
        _fa_bwd(qk[:, :, :H], qk[:, :, H:], v, o, lse, do, g4[:, :, :H], g4[:, :, H:H + Hkv], g4[:, :, H + Hkv:],
                ctx.job)
        L.call("pa_rope_rows", L.ptr(g), W, L.ptr(cos), L.ptr(sin), L.ptr(g), W, B * S, S, H + Hkv, D,
               int(ctx.neox) | 2, L.dcode(g), L.stream_ptr())
        return g, None, None, None, None, None, None, None, None


@static_op
def qkv_rope_attention(t, cos, sin, num_heads, num_kv_heads, head_dim, causal=True, scale=None, neox=True, groups=1):
    """Fused projection output t [B, S, (H + 2*Hkv) * D] -> attention(RoPE(q), RoPE(k), v) [B, S, H, D] with cos /
    sin the fp32 [S, D] tables of these positions. The HIP path (bf16/fp16, D in {64, 128, 256}) hands the whole
    qkv gradient back as one buffer; elsewhere it is the split + apply_rotary + flash_attention composition.
    ``groups`` > 1: the width holds ``groups`` consecutive [q | k | v] blocks of H/groups and Hkv/groups heads (the
    layout whose column-parallel shards are each one whole block: tensor-parallel rank r computes its heads from
    its own shard with groups = 1)."""
    H, Hkv, D, g = int(num_heads), int(num_kv_heads), int(head_dim), int(groups)
    B, S, W = t.shape
    if W != (H + 2 * Hkv) * D or H % Hkv or H % g or Hkv % g:
        raise ValueError(f"qkv_rope_attention: width {W} != (H + 2*Hkv) * D = {(H + 2 * Hkv) * D} "
                         f"(H={H}, Hkv={Hkv}, groups={g})")
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    cos = cos.float().contiguous()
    sin = sin.float().contiguous()
    if g > 1:  # regroup [q_0 k_0 v_0 | q_1 k_1 v_1 | ...] into one [q | k | v] layout
        Hg, Kg = H // g, Hkv // g
        tg = t.reshape(B, S, g, (Hg + 2 * Kg) * D)
        q = tg[..., :Hg * D].reshape(B, S, H * D)
        k = tg[..., Hg * D:(Hg + Kg) * D].reshape(B, S, Hkv * D)
        v = tg[..., (Hg + Kg) * D:].reshape(B, S, Hkv * D)
        t = torch.cat([q, k, v], -1)
    if (L.hip_enabled_for(t) and L.has("pa_rope_rows") and L.has("pa_flash_attn_fwd_ex")
            and t.dtype in (torch.bfloat16, torch.float16) and D in (64, 128, 256) and cos.shape[0] >= S
            and cos.shape[-1] == D):
        return _QKVRopeAttnHIP.apply(t, cos, sin, H, Hkv, D, bool(causal), scale, bool(neox))
    from .rope import apply_rotary
    q, k, v = t.split([H * D, Hkv * D, Hkv * D], -1)
    q = apply_rotary(q.reshape(B, S, H, D), cos, sin, neox)
    k = apply_rotary(k.reshape(B, S, Hkv, D), cos, sin, neox)
    return attention(q, k, v.reshape(B, S, Hkv, D), causal=causal, scale=scale)


def _padded_dim(D):
    """Head dims the kernel instantiates: 64, 128, 256; others (multiples of 8) are zero-padded up to one."""
    if D % 8 != 0 or D > 256:
        return None
    return 64 if D <= 64 else (128 if D <= 128 else 256)


def _hip_ok(q, k, v):
    if not L.hip_enabled_for(q) or not L.has("pa_flash_attn_fwd_ex"):
        return False
    if q.dtype not in (torch.bfloat16, torch.float16) or k.dtype != q.dtype or v.dtype != q.dtype:
        return False
    D = q.shape[-1]
    if _padded_dim(D) is None or k.shape[-1] != D or v.shape[-1] != D:
        return False
    return q.shape[-2] % k.shape[-2] == 0


@static_op
def flash_attention_qkvpacked(qkv, causal=True, scale=None, dropout=0.0, training=True):
    """qkv [B,S,H,3,D] -> [B,S,H,D]."""
    D = qkv.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    q, k, v = qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2]
    if _hip_ok(q, k, v) and D in (64, 128, 256) and not (dropout > 0 and training) and _lastdim_contig(qkv):
        return _FlashAttnQKVPackedHIP.apply(qkv, bool(causal), scale)
    return flash_attention(q, k, v, causal=causal, scale=scale, dropout=dropout, training=training)


def attention(q, k, v, causal=False, scale=None, mask=None, startend_row_indices=None, dropout=0.0, training=True,
              seed=None, cu_seqlens_q=None, cu_seqlens_k=None, max_seqlen_q=None, max_seqlen_k=None,
              return_lse=False):
    """Attention with every optional term on the HIP kernel: q/k/v [B,S,H,D] (or packed [total, H, D] with
    cu_seqlens), bool / additive ``mask`` broadcastable to [B, H, Sq, Sk], flashmask ``startend_row_indices``,
    in-kernel dropout, GQA, head dims up to 256. Returns o (and the fp32 log-sum-exp when ``return_lse``:
    [B, H, Sq], or [H, total_q] for varlen)."""
    varlen = cu_seqlens_q is not None
    D = q.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    p = float(dropout) if training else 0.0
    if varlen and (mask is not None or startend_row_indices is not None):
        raise ValueError("varlen attention takes no dense mask / flashmask (cu_seqlens define the sequences)")
    if mask is not None and startend_row_indices is not None:
        raise ValueError("pass either a dense mask or startend_row_indices, not both")
    if _hip_ok(q, k, v):
        Dp = _padded_dim(D)
        if Dp != D:
            q, k, v = (F.pad(t, (0, Dp - D)) for t in (q, k, v))
        if p > 0 and seed is None:
            seed = _draw_seed()
        job = _Job(q, k, varlen, causal, scale, mask, startend_row_indices, p, seed or 0, cu_seqlens_q, cu_seqlens_k,
                   max_seqlen_q, max_seqlen_k)
        o, lse = _FlashAttnHIP.apply(q, k, v, job)
        if Dp != D:
            o = o[..., :D]
        return (o, lse) if return_lse else o
    # CPU / uncovered dtypes: the math path, per sequence for varlen
    if varlen:
        cq, ck = cu_seqlens_q.tolist(), cu_seqlens_k.tolist()
        outs, lses = [], []
        for i in range(len(cq) - 1):
            qi, ki, vi = q[cq[i]:cq[i + 1]][None], k[ck[i]:ck[i + 1]][None], v[ck[i]:ck[i + 1]][None]
            outs.append(_sdpa(qi, ki, vi, causal, scale, None, p, training)[0])
            if return_lse:
                lses.append(_lse_reference(qi, ki, causal, scale, None)[0])
        o = torch.cat(outs, 0)
        return (o, torch.cat(lses, -1)) if return_lse else o
    if startend_row_indices is not None:
        mask = flashmask_keep(startend_row_indices, q.shape[1], k.shape[1], causal, q.device)
        causal = False
    o = _sdpa(q, k, v, causal, scale, mask, p, training)
    return (o, _lse_reference(q, k, causal, scale, mask)) if return_lse else o


def _lse_reference(q, k, causal, scale, mask):
    H, Hk = q.shape[2], k.shape[2]
    qf, kf = q.float().transpose(1, 2), k.float().transpose(1, 2)
    if Hk != H:
        kf = kf.repeat_interleave(H // Hk, 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Sq, Sk = q.shape[1], k.shape[1]
    if causal:
        s = s.masked_fill(~torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq), float("-inf"))
    if mask is not None:
        s = s.masked_fill(~mask, float("-inf")) if mask.dtype == torch.bool else s + mask.float()
    return torch.logsumexp(s, -1)


def flashmask_keep(startend, Sq, Sk, causal, device):
    """Boolean keep-mask [B, H|1, Sq, Sk] from startend_row_indices [B, H|1, Sk, n] (n = 1, 2 or 4): the dense
    form of the row intervals the kernel evaluates in place (reference semantics:
    python/paddle/nn/functional/flash_attention.py:1306 flashmask_attention)."""
    se = startend.to(torch.int64)
    rows = torch.arange(Sq, device=device).view(1, 1, Sq, 1)
    n = se.shape[-1]
    lts = se[..., 0].unsqueeze(2)
    if causal:
        lte = se[..., 1].unsqueeze(2) if n >= 2 else torch.full_like(lts, 1 << 40)
        masked = (rows >= lts) & (rows < lte)
        keep = ~masked & (rows >= torch.arange(Sk, device=device).view(1, 1, 1, Sk) - (Sk - Sq))
    else:
        if n == 2:
            lte = torch.full_like(lts, 1 << 40)
            ute = se[..., 1].unsqueeze(2)
            uts = torch.zeros_like(ute)
        else:
            lte, uts, ute = (se[..., i].unsqueeze(2) for i in (1, 2, 3))
        masked = ((rows >= lts) & (rows < lte)) | ((rows >= uts) & (rows < ute))
        keep = ~masked
    return keep


@static_op
def flash_attention(q, k, v, causal=False, scale=None, mask=None, dropout=0.0, training=True):
    """Attention over [B,S,H,D] tensors; returns [B,Sq,H,D]."""
    return attention(q, k, v, causal=causal, scale=scale, mask=mask, dropout=dropout, training=training)


def paged_decode_reference(q, key_cache, value_cache, block_tables, lens, scale=None):
    """fp32 reference: q [N,H,D]; caches [num_blocks,Hkv,bs,D]; block_tables [N,max_blocks]; lens [N]
    (cached tokens per sequence, the current one included). Returns [N,H,D] in q's dtype."""
    N, H, D = q.shape
    _, Hkv, bs, _ = key_cache.shape
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    nblk = block_tables.shape[1]
    tab = block_tables.long()
    K = key_cache[tab].permute(0, 2, 1, 3, 4).reshape(N, Hkv, nblk * bs, D).float()
    V = value_cache[tab].permute(0, 2, 1, 3, 4).reshape(N, Hkv, nblk * bs, D).float()
    G = H // Hkv
    qf = q.float().view(N, Hkv, G, D)
    s = torch.einsum("nkgd,nkld->nkgl", qf, K) * scale
    valid = torch.arange(nblk * bs, device=q.device)[None] < lens.long()[:, None]
    s = s.masked_fill(~valid[:, None, None], float("-inf"))
    o = torch.einsum("nkgl,nkld->nkgd", torch.softmax(s, -1), V)
    return o.reshape(N, H, D).to(q.dtype)


def _decode_splits(N, Hkv, max_len, bs):
    """Flash-decoding split count: enough workgroups to fill 256 CUs (≈4 per CU), but every split
    keeps ≥ 4 cache blocks so each of the workgroup's 4 waves has a block to stream."""
    nblk = max(1, (max_len + bs - 1) // bs)
    want = max(1, -(-1024 // max(1, N * Hkv)))
    return int(max(1, min(want, nblk // 4, 64)))


def _decode_hip_ok(q, key_cache, value_cache, Hkv):
    N, H, D = q.shape
    return (L.hip_enabled_for(q) and L.has("pa_paged_decode_attn") and q.dtype == torch.bfloat16
            and key_cache.dtype == torch.bfloat16 and value_cache.dtype == torch.bfloat16 and D == 128
            and H % Hkv == 0 and H // Hkv in (1, 2, 4, 8) and key_cache.is_contiguous()
            and value_cache.is_contiguous())


def _decode_launch(q, kc, vc, tables, lens, Hkv, bs, blk_stride, head_stride, scale, max_len):
    N, H, D = q.shape
    q = q.contiguous()
    tables = tables.to(torch.int32).contiguous()
    lens32 = lens.to(torch.int32).contiguous()
    max_blocks = tables.shape[1]
    splits = _decode_splits(N, Hkv, max_len, bs)
    part_o = torch.empty(N * H * splits * D, dtype=torch.float32, device=q.device)
    part_ml = torch.empty(N * H * splits * 2, dtype=torch.float32, device=q.device)
    out = torch.empty_like(q)
    L.call("pa_paged_decode_attn", L.ptr(q), L.ptr(kc), L.ptr(vc), L.ptr(tables), L.ptr(lens32), L.ptr(part_o),
           L.ptr(part_ml), L.ptr(out), N, H, Hkv, D, bs, max_blocks, splits, int(blk_stride), int(head_stride),
           float(scale), L.stream_ptr())
    return out


@static_op
def attention_bhsd(q, k, v, scale=None, mask=None, causal=False):
    """softmax(q k^T * scale (+ mask)) v over [B, H, S, D] tensors (the math-attention layout of traced programs),
    on the flash-attention kernel: the target of the fuse_dot_product_attention program pass. Returns [B, H, Sq, D]."""
    o = attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), causal=causal, scale=scale, mask=mask)
    return o.transpose(1, 2)


@static_op
def paged_decode_attention(q, key_cache, value_cache, block_tables, lens, scale=None, max_len=None):
    """One-token-per-sequence attention over a paged KV cache (block_multihead_attention decode).
    q [N,H,D]; caches [num_blocks,Hkv,block_size,D]; block_tables [N,max_blocks]; lens [N] cached
    tokens incl. the current one. HIP flash-decoding kernel (csrc/kernels/decode_attn.hip) for bf16,
    head_dim 128; otherwise the fp32 reference. ``max_len`` bounds lens (host hint for the split count;
    defaults to the block-table capacity, so no device sync)."""
    N, H, D = q.shape
    _, Hkv, bs, _ = key_cache.shape
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    if not _decode_hip_ok(q, key_cache, value_cache, Hkv):
        return paged_decode_reference(q, key_cache, value_cache, block_tables, lens, scale)
    ml = block_tables.shape[1] * bs if max_len is None else int(max_len)
    return _decode_launch(q, key_cache, value_cache, block_tables, lens, Hkv, bs, Hkv * bs * D, bs * D, scale, ml)


_VBLK = 64  # virtual block size when a dense cache is streamed by the paged kernel


_DENSE_TABLES = {}


@static_op
def dense_decode_attention(q, key_cache, value_cache, lens, scale=None, max_len=None):
    """Decode attention over a dense per-sequence cache [B,Hkv,max_len,D] (masked_multihead_attention
    layout). The same HIP kernel streams it as virtual 64-token blocks: block j of sequence b starts at
    b*Hkv*max_len*D + j*64*D and heads are max_len*D apart, so the block table is just b*Hkv*nb + j."""
    N, H, D = q.shape
    B, Hkv, Lc, _ = key_cache.shape
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    if not _decode_hip_ok(q, key_cache, value_cache, Hkv) or Lc % _VBLK != 0:
        valid = torch.arange(Lc, device=q.device)[None] < lens.long()[:, None]
        G = H // Hkv
        s = torch.einsum("nkgd,nkld->nkgl", q.float().view(N, Hkv, G, D), key_cache.float()) * scale
        s = s.masked_fill(~valid[:, None, None], float("-inf"))
        o = torch.einsum("nkgl,nkld->nkgd", torch.softmax(s, -1), value_cache.float())
        return o.reshape(N, H, D).to(q.dtype)
    nb = Lc // _VBLK
    key = (N, Hkv, nb, q.device)
    tables = _DENSE_TABLES.get(key)
    if tables is None:  # identical for every layer / step: built once (also outside any captured graph)
        tables = (torch.arange(N, device=q.device, dtype=torch.int32)[:, None] * (Hkv * nb)
                  + torch.arange(nb, device=q.device, dtype=torch.int32)[None])
        if len(_DENSE_TABLES) > 64:
            _DENSE_TABLES.clear()
        _DENSE_TABLES[key] = tables
    ml = Lc if max_len is None else int(max_len)
    return _decode_launch(q, key_cache, value_cache, tables, lens, Hkv, _VBLK, _VBLK * D, Lc * D, scale, ml)
