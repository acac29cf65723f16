"""LLaMA / LLaMA-2 / LLaMA-3 decoder (PaddleNLP-style llama modeling) on the MI355X hot-op set.

Reference: the reference's auto-parallel llama test models (test/auto_parallel/hybrid_strategy/
semi_auto_llama.py, test/deprecated/auto_parallel/auto_parallel_gpt_model.py for the shared
structure) and PaddleNLP's llama/modeling.py which the reference benchmarks.

MI355X mapping per block:
  * RMSNorm -> HIP wave-per-row kernel (ops.rms_norm)
  * fused QKV projection (one GEMM, [h, (H + 2*Hkv) * D]) -> RoPE HIP kernel on q/k
  * GQA flash attention -> HIP MFMA kernel (ops.flash_attention; K/V heads shared by H/Hkv q heads)
  * fused gate/up projection (one GEMM, [h, 2*ffn]) -> SwiGLU HIP kernel reading both halves in place
  * tensor parallel: column-parallel QKV / gate-up, row-parallel o / down, vocab-parallel embedding +
    parallel cross-entropy (parallel/tensor_parallel.py)
Decoding keeps a preallocated per-layer KV cache sized for ``max_length`` (HBM-resident; 288 GB per
GPU holds the 70B cache for long contexts) and appends one position per step.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .. import nn
from .. import ops as _ops
from ..framework.tensor import _wrap
from ..nn import initializer as I


@dataclass
class LlamaConfig:
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    initializer_range: float = 0.02
    tie_word_embeddings: bool = False
    use_recompute: bool = False
    recompute_granularity: str = "full"  # full (decoder layer) | full_attn (attention block) | core_attn (attention core)
    no_recompute_layers: tuple = ()      # layer indices kept out of recompute (PaddleNLP no_recompute_layers)
    fused_qkv_attention: bool = True  # training attention as ops.qkv_rope_attention (one-buffer qkv gradient)
    # models/llama_auto.py (PaddleNLP config names): one [q | k | v] projection / one [gate | up] projection per
    # tensor-parallel shard instead of separate linears
    fuse_attention_qkv: bool = False
    fuse_attention_ffn: bool = False
    tensor_parallel_degree: int = 1
    sequence_parallel: bool = False  # with TP: activations between the TP regions split over tokens (Megatron SP)
    sep_parallel_degree: int = 1  # segment parallelism: each rank of hcg's sep group holds S / sep tokens
    virtual_pp_degree: int = 1  # auto-parallel VPP: layer chunk c of pp * vpp goes to pp mesh c % pp (llama_auto)
    pad_token_id: int = 0
    bos_token_id: int = 1
    eos_token_id: int = 2
    # attention head width when it is not hidden_size / num_attention_heads (e.g. the tensor-parallel-local shape
    # of one rank: LLaMA-2 70B at TP 2 keeps hidden 8192 but 32 query heads of 128)
    attention_head_dim: int = 0

    @staticmethod
    def llama2_7b(**kw):
        return LlamaConfig(**kw)

    @staticmethod
    def llama2_13b(**kw):
        d = dict(hidden_size=5120, intermediate_size=13824, num_hidden_layers=40, num_attention_heads=40,
                 num_key_value_heads=40)
        d.update(kw)
        return LlamaConfig(**d)

    @staticmethod
    def llama2_70b(**kw):
        d = dict(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
                 num_key_value_heads=8)
        d.update(kw)
        return LlamaConfig(**d)

    @staticmethod
    def llama3_8b(**kw):
        d = dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                 num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192, rope_theta=500000.0,
                 bos_token_id=128000, eos_token_id=128001)
        d.update(kw)
        return LlamaConfig(**d)

    @staticmethod
    def tiny(**kw):
        d = dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=4,
                 num_key_value_heads=2, max_position_embeddings=256)
        d.update(kw)
        return LlamaConfig(**d)

    @property
    def head_dim(self):
        return self.attention_head_dim or self.hidden_size // self.num_attention_heads

    def num_params(self):
        h, f, L, V = self.hidden_size, self.intermediate_size, self.num_hidden_layers, self.vocab_size
        q = self.num_attention_heads * self.head_dim
        kv = self.num_key_value_heads * self.head_dim
        per = h * (q + 2 * kv) + q * h + 3 * h * f + 2 * h
        return L * per + V * h * (1 if self.tie_word_embeddings else 2) + h

    def flops_per_token(self, seq_len):
        q = self.num_attention_heads * self.head_dim
        return 6 * self.num_params() + 12 * self.num_hidden_layers * q * seq_len


def _tp():
    from ..parallel import tensor_parallel as tp
    return tp


def _sp():
    from ..parallel import sequence_parallel as sp
    return sp


def _use_sp(cfg):
    """Sequence parallelism (training, TP > 1): norms / residual adds on this rank's token block; the column
    linears all-gather the tokens overlapped with their GEMM, the row linears reduce-scatter them."""
    return bool(getattr(cfg, "sequence_parallel", False)) and cfg.tensor_parallel_degree > 1 \
        and cfg.sep_parallel_degree <= 1


class LlamaRMSNorm(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.weight = self.create_parameter([cfg.hidden_size], default_initializer=I.Constant(1.0))
        self.eps = cfg.rms_norm_eps
        if _use_sp(cfg):  # sees only this rank's tokens: its gradient is summed over the mp group per step
            _sp().mark_sequence_parallel(self.weight)

    def forward(self, x, residual=False):
        """``residual=True`` (pre-norm training blocks): returns (x_residual, rms_norm(x)) — use x_residual for the
        block's skip connection; on the HIP path its gradient is summed into this norm's input gradient by the
        backward kernel (ops.rms_norm_residual: no separate autograd accumulation add)."""
        if residual:
            r, h = _ops.rms_norm_residual(x._t, self.weight._t, self.eps)
            return _wrap(r), _wrap(h)
        return _wrap(_ops.rms_norm(x._t, self.weight._t, self.eps))

    def fuses_residual(self):
        """Whether forward(x, residual=True) is this layer's own math with nothing observing its output
        (subclasses overriding forward and layers with forward hooks keep the plain call)."""
        return (type(self).forward is LlamaRMSNorm.forward and not getattr(self, "_forward_pre_hooks", None)
                and not getattr(self, "_forward_post_hooks", None))


class _Rope:
    """Resident fp32 cos/sin tables, rebuilt only when a longer sequence or another device shows up."""

    def __init__(self, dim, base):
        self.dim, self.base = dim, base
        self.cos = self.sin = None

    def tables(self, n, device):
        if self.cos is None or self.cos.shape[0] < n or self.cos.device != device:
            m = max(n, 256)
            self.cos, self.sin = _ops.rope.rope_tables(m, self.dim, self.base, device=device, neox=True)
        return self.cos, self.sin


def _core(attn, fn, *ts):
    """The attention core ``fn(*ts)`` (torch tensors), checkpointed when the layer's recompute granularity is
    core_attn (``attn._rc_core``): only its inputs are kept, the core is re-run in backward."""
    if getattr(attn, "_rc_core", False):
        from ..distributed.fleet.recompute import recompute
        return recompute(lambda *a: _wrap(fn(*[x._t for x in a])), *[_wrap(x) for x in ts])._t
    return fn(*ts)


def _add_res(y, residual):
    return y if residual is None else _wrap(y._t + residual._t)


def _proj_res(layer, h, residual):
    """``layer(h) + residual``. For a plain hook-free linear (tp = 1) outside static tracing the add runs in the
    GEMM (ops.fused_linear residual=: the epilogue reads the residual, or hipBLASLt's C input) — no separate
    elementwise pass over the hidden states; its gradient is the output gradient itself."""
    if residual is None:
        return layer(h)
    w = layer.weight._t
    b = layer.bias._t if getattr(layer, "bias", None) is not None else None
    if (type(layer) is nn.Linear and not (layer._forward_pre_hooks or layer._forward_post_hooks)
            and h._t.dtype == w.dtype and residual._t.dtype == w.dtype and not _tracing()):
        return _wrap(_ops.fused_linear(h._t, w, b, residual=residual._t))
    return _wrap(layer(h)._t + residual._t)


def _tracing():
    from ..framework.trace_hook import _active_program
    return _active_program() is not None


class LlamaAttention(nn.Layer):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.tp = max(cfg.tensor_parallel_degree, 1)
        self.H = cfg.num_attention_heads // self.tp
        self.Hkv = max(cfg.num_key_value_heads // self.tp, 1)
        self.D = cfg.head_dim
        h = cfg.hidden_size
        out = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * self.D
        init = nn.ParamAttr(initializer=I.Normal(0.0, cfg.initializer_range))
        qw = cfg.num_attention_heads * self.D  # attention width (= h unless attention_head_dim is set)
        if self.tp > 1:
            tp = _tp()
            self.qkv_proj = tp.ColumnParallelLinear(h, out, weight_attr=init, has_bias=False, gather_output=False)
            self.o_proj = tp.RowParallelLinear(qw, h, weight_attr=init, has_bias=False, input_is_parallel=True)
        else:
            self.qkv_proj = nn.Linear(h, out, weight_attr=init, bias_attr=False)
            self.o_proj = nn.Linear(qw, h, weight_attr=init, bias_attr=False)
        self.rope = _Rope(self.D, cfg.rope_theta)

    def _qkv(self, x):
        t = self.qkv_proj(x)._t
        B, S = t.shape[0], t.shape[1]
        # per-rank layout [H | Hkv | Hkv] heads (column-parallel shards keep whole heads)
        q, k, v = t.split([self.H * self.D, self.Hkv * self.D, self.Hkv * self.D], -1)
        return q.view(B, S, self.H, self.D), k.view(B, S, self.Hkv, self.D), v.view(B, S, self.Hkv, self.D)

    def _forward_sp(self, x):
        """Sequence-parallel training: x is this rank's token block [B*S/mp, h]; the qkv projection all-gathers the
        tokens under its GEMM, the o projection reduce-scatters them back (parallel/sequence_parallel.py)."""
        sp = _sp()
        B, S = self.bs
        t = sp.column_sp_linear(x._t, self.qkv_proj.weight._t, None).view(B, S, -1)
        cos, sin = self.rope.tables(S, t.device)
        c, sn = cos[:S], sin[:S]
        o = _core(self, lambda tt: _ops.qkv_rope_attention(tt, c, sn, self.H, self.Hkv, self.D), t)
        return _wrap(sp.row_sp_linear(o.reshape(B * S, self.H * self.D), self.o_proj.weight._t))

    def forward(self, x, cache=None, pos=0, residual=None):
        """``residual``: return ``residual + attention output`` (the decoder's residual add, done by the
        o-projection GEMM on the plain training path — _proj_res)."""
        if cache is None and getattr(self, "bs", None) is not None and x._t.dim() == 2:
            return _add_res(self._forward_sp(x), residual)
        if cache is not None and isinstance(pos, torch.Tensor):
            return _add_res(self._decode_step(x, cache, pos), residual)
        if cache is None and self.cfg.sep_parallel_degree <= 1 and self.cfg.fused_qkv_attention:
            # training / full-sequence path: projection -> RoPE -> attention as one op whose backward returns the
            # whole qkv-projection gradient as one buffer (ops/attention.py qkv_rope_attention)
            t = self.qkv_proj(x)._t
            B, S = t.shape[0], t.shape[1]
            cos, sin = self.rope.tables(pos + S, t.device)
            c, sn = cos[pos:pos + S], sin[pos:pos + S]
            o = _core(self, lambda tt: _ops.qkv_rope_attention(tt, c, sn, self.H, self.Hkv, self.D), t)
            return _proj_res(self.o_proj, _wrap(o.reshape(B, S, self.H * self.D)), residual)
        q, k, v = self._qkv(x)
        B, S = q.shape[0], q.shape[1]
        if cache is None and self.cfg.sep_parallel_degree > 1:
            return _add_res(self._forward_sep(q, k, v, B, S), residual)
        cos, sin = self.rope.tables(pos + S, q.device)
        q = _ops.apply_rotary(q, cos[pos:pos + S], sin[pos:pos + S])
        k = _ops.apply_rotary(k, cos[pos:pos + S], sin[pos:pos + S])
        if cache is not None:
            # cache layout [B, Hkv, max_len, D] (the decode kernel's dense layout); prefill reads it back
            # as a strided [B, S, Hkv, D] view
            kc, vc = cache
            kc[:B, :, pos:pos + S].copy_(k.transpose(1, 2))
            vc[:B, :, pos:pos + S].copy_(v.transpose(1, 2))
            k, v = kc[:B, :, :pos + S].transpose(1, 2), vc[:B, :, :pos + S].transpose(1, 2)
            causal = S > 1
        else:
            causal = True
        o = _core(self, lambda qq, kk, vv: _ops.flash_attention(qq, kk, vv, causal=causal), q, k, v)
        return _proj_res(self.o_proj, _wrap(o.reshape(B, S, self.H * self.D)), residual)

    def _forward_sep(self, q, k, v, B, S):
        """Segment-parallel training step: this rank holds tokens [r * S, (r + 1) * S) of every sequence;
        RoPE uses the global positions and attention runs over the full sequence after a head / sequence
        all-to-all (parallel/segment_parallel.py)."""
        from ..distributed.fleet.topology import _get_hcg
        from ..parallel.segment_parallel import segment_attention
        g = _get_hcg().get_sep_parallel_group()
        off = g.rank * S
        cos, sin = self.rope.tables(off + S, q.device)
        q = _ops.apply_rotary(q, cos[off:off + S], sin[off:off + S])
        k = _ops.apply_rotary(k, cos[off:off + S], sin[off:off + S])
        o = segment_attention(q, k, v, g, causal=True)
        return self.o_proj(_wrap(o.reshape(B, S, self.H * self.D)))

    def _decode_step(self, x, cache, pos_t):
        """One token per sequence at the device-side position ``pos_t`` ([1] int64): no host value is
        read, so the step can be captured once into a hipGraph and replayed for every token. One fused
        kernel rotates Q/K with the RoPE rows at pos_t, splits the QKV projection and writes K/V into the
        dense cache at pos_t; attention is the flash-decoding HIP kernel over the first pos_t + 1 tokens."""
        kc, vc = cache
        t = self.qkv_proj(x)._t
        B = t.shape[0]
        q = t  # dtype / device carrier for the context below
        Lc = kc.shape[2]
        ctx = _DECODE_CTX.get(id(pos_t))
        if ctx is None or ctx[0] is not pos_t or ctx[1] != (Lc, B, q.device):
            # per-step constants shared by every layer (computed once per captured step, not per layer)
            cos, sin = self.rope.tables(Lc, q.device)
            ctx = (pos_t, (Lc, B, q.device), cos.index_select(0, pos_t), sin.index_select(0, pos_t),
                   (pos_t + 1).to(torch.int32).expand(B).contiguous())
            _DECODE_CTX.clear()
            _DECODE_CTX[id(pos_t)] = ctx
        _, _, cs, sn, lens = ctx
        q = _ops.decode_rope_cache(t.reshape(B, -1), self.H, self.Hkv, self.D, cs, sn, pos_t, kc, vc)
        o = _ops.dense_decode_attention(q, kc[:B], vc[:B], lens, max_len=Lc)
        return self.o_proj(_wrap(o.reshape(B, 1, self.H * self.D)))


# decode-step constants keyed by the position tensor; _decode_logits clears it at the start of each step
_DECODE_CTX = {}


class LlamaMLP(nn.Layer):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        h, f = cfg.hidden_size, cfg.intermediate_size
        self.tp = max(cfg.tensor_parallel_degree, 1)
        init = nn.ParamAttr(initializer=I.Normal(0.0, cfg.initializer_range))
        if self.tp > 1:
            tp = _tp()
            # gate/up interleaved per rank: each rank's shard holds [gate_r | up_r]
            self.gate_up_proj = tp.ColumnParallelLinear(h, 2 * f, weight_attr=init, has_bias=False, gather_output=False)
            self.down_proj = tp.RowParallelLinear(f, h, weight_attr=init, has_bias=False, input_is_parallel=True)
        else:
            self.gate_up_proj = nn.Linear(h, 2 * f, weight_attr=init, bias_attr=False)
            self.down_proj = nn.Linear(f, h, weight_attr=init, bias_attr=False)
        self.sp = _use_sp(cfg)

    def forward(self, x, residual=None):
        """``residual``: return ``residual + MLP output`` (added by the down-projection GEMM when it can be)."""
        if self.tp > 1 and x._t.dim() == 2 and getattr(self, "sp", False):  # sequence parallel: token block in / out
            sp = _sp()
            h = _ops.swiglu(sp.column_sp_linear(x._t, self.gate_up_proj.weight._t, None))
            return _add_res(_wrap(sp.row_sp_linear(h, self.down_proj.weight._t)), residual)
        # one-input swiglu: its backward writes d[gate | up] as one buffer (no chunk / cat in autograd)
        return _proj_res(self.down_proj, _wrap(_ops.swiglu(self.gate_up_proj(x)._t)), residual)


class LlamaDecoderLayer(nn.Layer):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.input_layernorm = LlamaRMSNorm(cfg)
        self.self_attn = LlamaAttention(cfg)
        self.post_attention_layernorm = LlamaRMSNorm(cfg)
        self.mlp = LlamaMLP(cfg)

    def forward(self, x, cache=None, pos=0):
        n1, n2 = self.input_layernorm, self.post_attention_layernorm
        if (cache is None and torch.is_grad_enabled() and isinstance(n1, LlamaRMSNorm) and n1.fuses_residual()
                and isinstance(n2, LlamaRMSNorm) and n2.fuses_residual()):
            # training: each residual branch's gradient is summed into the RMSNorm input gradient by the norm's
            # backward kernel (LlamaRMSNorm(residual=True) -> ops.rms_norm_residual, a recorded static op, so a
            # captured program keeps it) instead of autograd's separate accumulation add
            # the residual adds themselves run in the o / down projection GEMMs' epilogues (_proj_res)
            r, h = n1(x, residual=True)
            t = self._attn(h, cache, pos, residual=r)
            r, h = n2(t, residual=True)
            return self.mlp(h, residual=r)
        h = self._attn(self.input_layernorm(x), cache, pos)
        x = _wrap(x._t + h._t)
        h = self.mlp(self.post_attention_layernorm(x))
        return _wrap(x._t + h._t)

    def _attn(self, h, cache, pos, residual=None):
        """Self-attention under the layer's recompute granularity (LlamaModel sets ``_rc``): full_attn checkpoints
        the attention block (projections included), core_attn only the attention core. ``residual``: added to the
        output (by the o-projection GEMM outside full_attn recompute)."""
        g = getattr(self, "_rc", None) if cache is None else None
        if g == "full_attn":
            from ..distributed.fleet.recompute import recompute
            return _add_res(recompute(self.self_attn, h), residual)
        self.self_attn._rc_core = g == "core_attn"
        if residual is None:
            return self.self_attn(h, cache, pos)
        return self.self_attn(h, cache, pos, residual=residual)


class LlamaModel(nn.Layer):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        init = nn.ParamAttr(initializer=I.Normal(0.0, cfg.initializer_range))
        if cfg.tensor_parallel_degree > 1:
            self.embed_tokens = _tp().VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, weight_attr=init)
        else:
            self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size, weight_attr=init)
        self.layers = nn.LayerList([LlamaDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.norm = LlamaRMSNorm(cfg)

    def _forward_infer(self, x, caches, pos):
        """Inference layer loop with the residual adds fused into the following RMSNorm (one HIP pass for
        x += h; n = norm(x)), including across layer boundaries and into the final norm."""
        xt, h = x._t, None
        for i, layer in enumerate(self.layers):
            if h is None:
                n = _ops.rms_norm(xt, layer.input_layernorm.weight._t, layer.input_layernorm.eps)
            else:
                xt, n = _ops.add_rms_norm(xt, h, layer.input_layernorm.weight._t, layer.input_layernorm.eps,
                                          inplace=i > 0)
            a = layer.self_attn(_wrap(n), None if caches is None else caches[i], pos)._t
            xt, n = _ops.add_rms_norm(xt, a, layer.post_attention_layernorm.weight._t,
                                      layer.post_attention_layernorm.eps, inplace=i > 0)
            h = layer.mlp(_wrap(n))._t
        _, out = _ops.add_rms_norm(xt, h, self.norm.weight._t, self.norm.eps, inplace=True)
        return _wrap(out)

    def forward(self, input_ids, caches=None, pos=0):
        sp_on = _use_sp(self.config) and caches is None and self.training and torch.is_grad_enabled()
        B, S = input_ids.shape[0], input_ids.shape[-1]
        for layer in self.layers:
            layer.self_attn.bs = (B, S) if sp_on else None
        self.sp_bs = (B, S) if sp_on else None
        if sp_on:  # this rank's token block: the vocab-parallel partial embeddings reduce-scattered over tokens
            emb = self.embed_tokens.local_lookup(input_ids._t).reshape(B * S, -1)
            x = _wrap(_sp().reduce_scatter_tokens(emb))
        else:
            x = self.embed_tokens(input_ids)
            if not torch.is_grad_enabled() and len(self.layers) > 0 and x._t.is_cuda:
                return self._forward_infer(x, caches, pos)
        rc = self.config.use_recompute and self.training and caches is None
        gran = self.config.recompute_granularity
        skip = set(self.config.no_recompute_layers or ())
        if rc:
            from ..distributed.fleet.recompute import recompute
        for i, layer in enumerate(self.layers):
            on = rc and i not in skip
            if on and gran == "full":
                x = recompute(layer, x)
            else:
                layer._rc = gran if on else None  # full_attn / core_attn: the layer checkpoints part of itself
                x = layer(x, None if caches is None else caches[i], pos)
        return self.norm(x)


class LlamaForCausalLM(nn.Layer):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        self.llama = LlamaModel(cfg)
        if not cfg.tie_word_embeddings:
            tp = max(cfg.tensor_parallel_degree, 1)
            self.lm_head_weight = self.create_parameter([cfg.vocab_size // tp, cfg.hidden_size],
                                                        default_initializer=I.Normal(0.0, cfg.initializer_range))
            if tp > 1:
                self.lm_head_weight.is_distributed = True

    def _logits(self, h):
        w = self.llama.embed_tokens.weight if self.config.tie_word_embeddings else self.lm_head_weight
        ht = h._t if h._t.dtype == w._t.dtype else h._t.to(w._t.dtype)
        bs = getattr(getattr(self, "llama", None), "sp_bs", None)  # (the pipeline head shares this method)
        if bs is not None and ht.dim() == 2:
            # token blocks -> vocab-parallel logits of all tokens (the token all-gather overlaps the GEMM)
            return _wrap(_sp().column_sp_linear_nt(ht, w._t).view(bs[0], bs[1], -1))
        if self.config.tensor_parallel_degree > 1:
            ht = _tp().c_identity(ht)
        return _wrap(torch.matmul(ht, w._t.t()))

    def forward(self, input_ids, caches=None, pos=0):
        return self._logits(self.llama(input_ids, caches, pos))

    # ------------------------------------------------------------------ generation
    def new_cache(self, batch, max_length):
        cfg = self.config
        p = next(iter(self.parameters()))
        Hkv = max(cfg.num_key_value_heads // max(cfg.tensor_parallel_degree, 1), 1)
        max_length = -(-max_length // 64) * 64  # whole 64-token blocks for the decode kernel
        shape = (batch, Hkv, max_length, cfg.head_dim)
        return [(torch.zeros(shape, dtype=p._t.dtype, device=p._t.device),
                 torch.zeros(shape, dtype=p._t.dtype, device=p._t.device)) for _ in range(cfg.num_hidden_layers)]

    @torch.no_grad()
    def generate(self, input_ids, max_new_tokens=16, decode_strategy="greedy_search", temperature=1.0, top_k=0,
                 top_p=1.0, eos_token_id=None, use_graph=False):
        """Prefill once, then one token per step against the KV cache. Returns (ids, scores).
        ``use_graph`` (greedy, HIP device): the decode step is captured once into a hipGraph and replayed
        per token — decode is launch-bound at serving batch sizes, the graph turns ~15 launches per layer
        into one submission per token."""
        ids = input_ids._t
        B, S = ids.shape
        if use_graph and decode_strategy == "greedy_search" and ids.is_cuda:
            return self._generate_graph(ids, max_new_tokens, eos_token_id)
        caches = self.new_cache(B, S + max_new_tokens)
        logits = self.forward(_wrap(ids), caches, 0)._t[:, -1].float()
        out, scores = [], []
        eos = self.config.eos_token_id if eos_token_id is None else eos_token_id
        done = torch.zeros(B, dtype=torch.bool, device=ids.device)
        for t in range(max_new_tokens):
            if decode_strategy == "sampling":
                lg = logits / max(temperature, 1e-5)
                if top_k:
                    kth = lg.topk(top_k, -1).values[:, -1:]
                    lg = lg.masked_fill(lg < kth, float("-inf"))
                probs = torch.softmax(lg, -1)
                if top_p < 1.0:
                    sp, si = probs.sort(-1, descending=True)
                    keep = sp.cumsum(-1) - sp <= top_p
                    probs = torch.zeros_like(probs).scatter_(-1, si, sp * keep)
                    probs = probs / probs.sum(-1, keepdim=True)
                nxt = torch.multinomial(probs, 1).squeeze(-1)
            else:
                nxt = logits.argmax(-1)
            scores.append(torch.log_softmax(logits, -1).gather(-1, nxt[:, None]).squeeze(-1))
            nxt = torch.where(done, torch.full_like(nxt, self.config.pad_token_id), nxt)
            out.append(nxt)
            done |= nxt == eos
            if bool(done.all()) or t == max_new_tokens - 1:
                break
            logits = self.forward(_wrap(nxt[:, None]), caches, S + t)._t[:, -1].float()
        return _wrap(torch.stack(out, 1)), _wrap(torch.stack(scores, 1))


    def _decode_logits(self, tok, caches, pos_t):
        _DECODE_CTX.clear()  # recompute the per-step RoPE rows / lengths once, in this step (and graph)
        x = self.llama.embed_tokens(_wrap(tok))
        if not torch.is_grad_enabled() and x._t.is_cuda:
            return self._logits(self.llama._forward_infer(x, caches, pos_t))._t[:, -1].float()
        for i, layer in enumerate(self.llama.layers):
            x = layer(x, caches[i], pos_t)
        return self._logits(self.llama.norm(x))._t[:, -1].float()

    def _generate_graph(self, ids, max_new_tokens, eos_token_id):
        B, S = ids.shape
        caches = self.new_cache(B, S + max_new_tokens)
        logits = self.forward(_wrap(ids), caches, 0)._t[:, -1].float()
        eos = self.config.eos_token_id if eos_token_id is None else eos_token_id
        tok = torch.empty(B, 1, dtype=ids.dtype, device=ids.device)
        pos_t = torch.zeros(1, dtype=torch.int64, device=ids.device)
        out, scores = [], []
        done = torch.zeros(B, dtype=torch.bool, device=ids.device)

        def take(lg):
            nxt = lg.argmax(-1)
            scores.append(torch.log_softmax(lg, -1).gather(-1, nxt[:, None]).squeeze(-1))
            nxt = torch.where(done, torch.full_like(nxt, self.config.pad_token_id), nxt)
            out.append(nxt)
            done.logical_or_(nxt == eos)
            return nxt

        nxt = take(logits)
        if max_new_tokens > 1:
            tok.copy_(nxt[:, None])
            pos_t.fill_(S)
            # warm up once eagerly on a side stream (allocator / kernel choices settle), then capture
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._decode_logits(tok, caches, pos_t)
            torch.cuda.current_stream().wait_stream(s)
            from ..device.cuda.graphs import CUDAGraph, capture
            g = CUDAGraph()
            with capture(g):
                static_logits = self._decode_logits(tok, caches, pos_t)
            for t in range(1, max_new_tokens):
                tok.copy_(nxt[:, None])
                pos_t.fill_(S + t - 1)
                g.replay()
                nxt = take(static_logits)
        return _wrap(torch.stack(out, 1)), _wrap(torch.stack(scores, 1))


class LlamaPretrainingCriterion(nn.Layer):
    def __init__(self, cfg: LlamaConfig = None, ignore_index=-100):
        super().__init__()
        self.cfg = cfg
        self.ignore_index = ignore_index

    def forward(self, logits, labels):
        lt = logits._t
        if self.cfg is not None and self.cfg.tensor_parallel_degree > 1:
            per_tok = _tp().parallel_cross_entropy_raw(lt, labels._t, self.ignore_index)
        else:
            per_tok = _ops.softmax_cross_entropy(lt, labels._t, self.ignore_index)
        valid = (labels._t != self.ignore_index).sum().clamp_min(1)
        return _wrap(per_tok.sum() / valid)


# ----------------------------------------------------------------------------------------- pipeline
class LlamaEmbeddingPipe(nn.Layer):
    """First pipeline segment: token ids -> hidden states (vocab-parallel under TP)."""

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        init = nn.ParamAttr(initializer=I.Normal(0.0, cfg.initializer_range))
        if cfg.tensor_parallel_degree > 1:
            self.embed_tokens = _tp().VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, weight_attr=init)
        else:
            self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size, weight_attr=init)

    def forward(self, input_ids):
        return self.embed_tokens(input_ids)


class LlamaDecoderLayerPipe(LlamaDecoderLayer):
    def forward(self, x):
        return super().forward(x)


class LlamaHeadPipe(nn.Layer):
    """Last pipeline segment: final RMSNorm + LM head (vocab-sharded logits under TP)."""

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        self.norm = LlamaRMSNorm(cfg)
        tp = max(cfg.tensor_parallel_degree, 1)
        self.lm_head_weight = self.create_parameter([cfg.vocab_size // tp, cfg.hidden_size],
                                                    default_initializer=I.Normal(0.0, cfg.initializer_range))
        if tp > 1:
            self.lm_head_weight.is_distributed = True

    def forward(self, x):
        h = self.norm(x)
        w = self.lm_head_weight
        ht = h._t if h._t.dtype == w._t.dtype else h._t.to(w._t.dtype)
        bs = getattr(getattr(self, "llama", None), "sp_bs", None)  # (the pipeline head shares this method)
        if bs is not None and ht.dim() == 2:
            # token blocks -> vocab-parallel logits of all tokens (the token all-gather overlaps the GEMM)
            return _wrap(_sp().column_sp_linear_nt(ht, w._t).view(bs[0], bs[1], -1))
        if self.config.tensor_parallel_degree > 1:
            ht = _tp().c_identity(ht)
        return _wrap(torch.matmul(ht, w._t.t()))


def LlamaForCausalLMPipe(cfg: LlamaConfig, num_stages=None, num_virtual_pipeline_stages=None, seg_method="uniform",
                         recompute_interval=0):
    """LLaMA as a PipelineLayer (reference: PaddleNLP LlamaForCausalLMPipe, built from LayerDescs):
    [embedding] + L x [decoder layer] + [norm + lm head], loss = LlamaPretrainingCriterion. Composes with
    tensor parallelism (cfg.tensor_parallel_degree) and interleaved virtual stages: the PP4 x TP2 layout of
    the 70B config puts 20 decoder layers and 8.75B parameters on each MI355X."""
    from ..parallel.pipeline import LayerDesc, PipelineLayer
    if _use_sp(cfg):
        raise NotImplementedError("LlamaForCausalLMPipe: sequence_parallel is implemented on LlamaForCausalLM "
                                  "(fleet tensor parallelism without the pipeline layer)")
    descs = [LayerDesc(LlamaEmbeddingPipe, cfg)]
    descs += [LayerDesc(LlamaDecoderLayerPipe, cfg) for _ in range(cfg.num_hidden_layers)]
    descs.append(LayerDesc(LlamaHeadPipe, cfg))
    return PipelineLayer(descs, num_stages=num_stages, loss_fn=LlamaPretrainingCriterion(cfg), seg_method=seg_method,
                         recompute_interval=recompute_interval,
                         num_virtual_pipeline_stages=num_virtual_pipeline_stages)
