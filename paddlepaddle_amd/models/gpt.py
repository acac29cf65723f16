"""GPT-3 family (1.3B / 6.7B / 13B / 175B shapes) — the flagship training model.

Reference model: test/deprecated/auto_parallel/auto_parallel_gpt_model.py:602 (GPTModel),
:740 (GPTForPretraining), :829 (GPTPretrainingCriterion); PaddleNLP gpt3 configs (pre-LN, GELU,
learned absolute positions, tied input/output embedding).

MI355X-native layer (per decoder block):
  LN (HIP norm kernel) → fused QKV GEMM (hipBLASLt, bias in epilogue) → flash attention on
  [B,S,H,D] views of the QKV buffer (HIP MFMA kernel, causal) → out-proj GEMM → dropout+residual
  → LN → FFN1 GEMM + fused bias-GELU (HIP) → FFN2 GEMM → dropout+residual.
Tensor parallel (mp_degree>1): QKV/FFN1 column-parallel, out-proj/FFN2 row-parallel, vocab-parallel
embedding + parallel cross-entropy (parallel/tensor_parallel.py). With ``sequence_parallel`` the hidden states
between the TP regions are token shards [B*S/mp, H]: LayerNorm / dropout / residual on the shard, all-gather /
reduce-scatter overlapped with the GEMMs (parallel/sequence_parallel.py). Activation recompute per block.
"""
from __future__ import annotations

import dataclasses
import math

import torch

from .. import nn
from ..framework.tensor import Tensor, _wrap
from ..nn import functional as F
from ..nn import initializer as I
from .. import ops as _ops


@dataclasses.dataclass
class GPTConfig:
    vocab_size: int = 50304
    hidden_size: int = 5120
    num_hidden_layers: int = 40
    num_attention_heads: int = 40
    intermediate_size: int = 20480
    max_position_embeddings: int = 2048
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.0
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-5
    tie_word_embeddings: bool = True
    use_recompute: bool = False
    recompute_granularity: str = "full"  # full (decoder layer) | full_attn (attention block) | core_attn
    no_recompute_layers: tuple = ()       # layer indices kept out of recompute
    tensor_parallel_degree: int = 1
    sequence_parallel: bool = False
    fuse_attention_qkv: bool = True
    # LM head + CE over vocabulary slices (ops/lm_head.py): the [tokens, vocab] logits are never materialised
    fused_head_ce: bool = False

    @staticmethod
    def gpt3_13b(**kw):
        return GPTConfig(**kw)

    @staticmethod
    def gpt3_6_7b(**kw):
        d = dict(hidden_size=4096, num_hidden_layers=32, num_attention_heads=32, intermediate_size=16384)
        d.update(kw)
        return GPTConfig(**d)

    @staticmethod
    def gpt3_1_3b(**kw):
        d = dict(hidden_size=2048, num_hidden_layers=24, num_attention_heads=16, intermediate_size=8192)
        d.update(kw)
        return GPTConfig(**d)

    @staticmethod
    def gpt3_175b(**kw):
        d = dict(hidden_size=12288, num_hidden_layers=96, num_attention_heads=96, intermediate_size=49152)
        d.update(kw)
        return GPTConfig(**d)

    @staticmethod
    def tiny(**kw):
        d = dict(vocab_size=512, hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=512,
                 max_position_embeddings=128, hidden_dropout_prob=0.0)
        d.update(kw)
        return GPTConfig(**d)

    def num_params(self):
        h, L, f, V, P = (self.hidden_size, self.num_hidden_layers, self.intermediate_size, self.vocab_size,
                         self.max_position_embeddings)
        per_layer = 4 * h * h + 4 * h + 2 * h * f + f + h + 4 * h
        return L * per_layer + V * h + P * h + 2 * h

    def flops_per_token(self, seq_len, recompute=False):
        """Training FLOPs per token: 6N (fwd+bwd GEMMs) + causal attention scores; +2N with full recompute."""
        n = self.num_params() - self.max_position_embeddings * self.hidden_size
        # QK^T + PV, forward + backward = 12 L h S per token for full attention; a causal mask does half of it
        attn = 6 * self.num_hidden_layers * self.hidden_size * seq_len
        f = 6 * n + attn
        if recompute:
            f += 2 * n + attn / 3
        return f


def _tp():
    from ..parallel import tensor_parallel as tp
    return tp


def _sp():
    from ..parallel import sequence_parallel as sp
    return sp


def _use_sp(cfg):
    return cfg.sequence_parallel and cfg.tensor_parallel_degree > 1


class GPTEmbeddings(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        init = I.Normal(0.0, cfg.initializer_range)
        if cfg.tensor_parallel_degree > 1:
            self.word_embeddings = _tp().VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size,
                                                                weight_attr=nn.ParamAttr(initializer=init))
        else:
            self.word_embeddings = nn.Embedding(cfg.vocab_size, cfg.hidden_size,
                                                weight_attr=nn.ParamAttr(initializer=init))
        self.position_embeddings = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size,
                                                weight_attr=nn.ParamAttr(initializer=init))
        self.dropout = nn.Dropout(cfg.hidden_dropout_prob)

        self.sp = _use_sp(cfg)
        if self.sp:
            _sp().mark_sequence_parallel(self.position_embeddings.weight)

    def forward(self, input_ids, position_ids=None):
        if self.sp:
            return self._forward_sp(input_ids, position_ids)
        if position_ids is None:
            S = input_ids.shape[-1]
            position_ids = _wrap(torch.arange(S, device=input_ids._t.device).unsqueeze(0))
        x = self.word_embeddings(input_ids)._t
        pe = self.position_embeddings(position_ids)._t
        p = self.dropout.p if self.training else 0.0
        return _wrap(_ops.dropout_add(x + pe, None, p, self.training))

    def _forward_sp(self, input_ids, position_ids):
        """This rank's token block [B*S/mp, H]: the vocab-parallel partial embeddings are reduce-scattered over
        tokens (half the bytes of the all-reduce), positions are looked up for the block's own tokens."""
        sp = _sp()
        ids = input_ids._t
        B, S = ids.shape[0], ids.shape[-1]
        emb = self.word_embeddings.local_lookup(ids).reshape(B * S, -1)
        x = sp.reduce_scatter_tokens(emb)
        r0, r1 = sp.token_block_range(B * S)
        if position_ids is None:
            pos = torch.arange(r0, r1, device=ids.device) % S
        else:
            pos = position_ids._t.expand(B, S).reshape(-1)[r0:r1]
        pe = torch.nn.functional.embedding(pos, self.position_embeddings.weight._t)
        p = self.dropout.p if self.training else 0.0
        return _wrap(_ops.dropout_add(x + pe, None, p, self.training))


class GPTAttention(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        h = cfg.hidden_size
        self.num_heads = cfg.num_attention_heads
        self.head_dim = h // self.num_heads
        self.tp = cfg.tensor_parallel_degree
        init = I.Normal(0.0, cfg.initializer_range)
        out_init = I.Normal(0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_hidden_layers))
        if self.tp > 1:
            tp = _tp()
            self.qkv_proj = tp.ColumnParallelLinear(h, 3 * h, weight_attr=nn.ParamAttr(initializer=init),
                                                    has_bias=True, gather_output=False)
            self.out_proj = tp.RowParallelLinear(h, h, weight_attr=nn.ParamAttr(initializer=out_init),
                                                 has_bias=True, input_is_parallel=True)
            self.local_heads = self.num_heads // self.tp
        else:
            self.qkv_proj = nn.Linear(h, 3 * h, weight_attr=nn.ParamAttr(initializer=init))
            self.out_proj = nn.Linear(h, h, weight_attr=nn.ParamAttr(initializer=out_init))
            self.local_heads = self.num_heads
        self.attn_dropout = cfg.attention_probs_dropout_prob
        self.sp = _use_sp(cfg)
        self.bs = None  # (B, S) of the current micro-batch (sequence parallel: x is a token block)
        if self.sp:
            _sp().mark_sequence_parallel(self.out_proj.bias)

    def forward(self, x):
        if self.sp:
            return self._forward_sp(x)
        qkv = self.qkv_proj(x)._t  # [B, S, 3*h_local]
        B, S = qkv.shape[0], qkv.shape[1]
        qkv = qkv.view(B, S, self.local_heads, 3, self.head_dim)
        o = self._core(qkv)
        o = o.reshape(B, S, self.local_heads * self.head_dim)
        return self.out_proj(_wrap(o))

    def _core(self, qkv):
        """The attention core, checkpointed under recompute_granularity core_attn (``_rc_core``)."""
        def fn(t):
            return _ops.flash_attention_qkvpacked(t, causal=True, dropout=self.attn_dropout, training=self.training)
        if getattr(self, "_rc_core", False):
            from ..distributed.fleet.recompute import recompute
            return recompute(lambda a: _wrap(fn(a._t)), _wrap(qkv))._t
        return fn(qkv)

    def _forward_sp(self, x):
        sp = _sp()
        B, S = self.bs
        w, b = self.qkv_proj.weight._t, self.qkv_proj.bias._t
        t = x._t if x._t.dtype == w.dtype else x._t.to(w.dtype)
        qkv = sp.column_sp_linear(t, w, b)  # [B*S, 3*h_local]: all-gather overlapped with the GEMM
        qkv = qkv.view(B, S, self.local_heads, 3, self.head_dim)
        o = _ops.flash_attention_qkvpacked(qkv, causal=True, dropout=self.attn_dropout, training=self.training)
        o = o.reshape(B * S, self.local_heads * self.head_dim)
        y = sp.row_sp_linear(o, self.out_proj.weight._t)  # GEMM pipelined with the reduce-scatter
        return _wrap(y + self.out_proj.bias._t)


def _tracing():
    """A static program is being traced (its passes / SPMD rules see the two linears, not the fused op)."""
    from ..framework.trace_hook import _active_program
    return _active_program() is not None


class GPTMLP(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        h, f = cfg.hidden_size, cfg.intermediate_size
        init = I.Normal(0.0, cfg.initializer_range)
        out_init = I.Normal(0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_hidden_layers))
        self.tp = cfg.tensor_parallel_degree
        if self.tp > 1:
            tp = _tp()
            self.linear1 = tp.ColumnParallelLinear(h, f, weight_attr=nn.ParamAttr(initializer=init), has_bias=True,
                                                   gather_output=False, fuse_bias_act="gelu")
            self.linear2 = tp.RowParallelLinear(f, h, weight_attr=nn.ParamAttr(initializer=out_init), has_bias=True,
                                                input_is_parallel=True)
        else:
            self.linear1 = nn.Linear(h, f, weight_attr=nn.ParamAttr(initializer=init))
            self.linear2 = nn.Linear(f, h, weight_attr=nn.ParamAttr(initializer=out_init))
        self.sp = _use_sp(cfg)
        if self.sp:
            _sp().mark_sequence_parallel(self.linear2.bias)

    def forward(self, x):
        if self.sp:
            sp = _sp()
            w1 = self.linear1.weight._t
            t = x._t if x._t.dtype == w1.dtype else x._t.to(w1.dtype)
            h = sp.column_sp_linear(t, w1, self.linear1.bias._t, act="gelu")
            y = sp.row_sp_linear(h, self.linear2.weight._t)
            return _wrap(y + self.linear2.bias._t)
        if self.tp > 1:
            h = self.linear1(x)
        else:
            w, b = self.linear1.weight._t, self.linear1.bias._t
            xt = x._t
            if xt.dtype != w.dtype:
                xt = xt.to(w.dtype)
            l2 = self.linear2
            w2, b2 = l2.weight._t, l2.bias._t
            if (w.dtype in (torch.bfloat16, torch.float16) and w2.dtype == w.dtype and b2.dtype == w.dtype
                    and not (l2._forward_pre_hooks or l2._forward_post_hooks or _tracing())):
                # fc1 -> GELU -> fc2 as one op: its backward runs the GELU backward (and fc1's bias gradient) in
                # fc2's data-gradient GEMM epilogue (ops/linear.py _FFNGeluFn)
                return _wrap(_ops.ffn_gelu(xt, w, b, w2, b2))
            h = _wrap(_ops.fused_linear(xt, w, b, act="gelu"))
        return self.linear2(h)


class GPTDecoderLayer(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.norm1 = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.self_attn = GPTAttention(cfg)
        self.norm2 = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.mlp = GPTMLP(cfg)
        self.dropout1 = nn.Dropout(cfg.hidden_dropout_prob)
        self.dropout2 = nn.Dropout(cfg.hidden_dropout_prob)
        if _use_sp(cfg):
            _sp().mark_sequence_parallel(self.norm1.weight, self.norm1.bias, self.norm2.weight, self.norm2.bias)

    def _ln(self, norm, x):
        """(residual, LN(x)): the residual's gradient is summed into the LN input gradient by the LN backward
        kernel (ops.layer_norm_residual) instead of a separate add."""
        r, h = _ops.layer_norm_residual(x._t, norm.weight._t, norm.bias._t, norm._epsilon)
        return r, _wrap(h)

    def _attn(self, h):
        """Self-attention under the layer's recompute granularity (GPTModel sets ``_rc``)."""
        return _gpt_attn(self, h)

    def forward(self, x):
        # residual + dropout fused in one HIP pass (mask regenerated from a seed in backward)
        p = self.dropout1.p if self.training else 0.0
        r, h = self._ln(self.norm1, x)
        x = _wrap(_ops.dropout_add(self._attn(h)._t, r, p, self.training))
        r, h = self._ln(self.norm2, x)
        x = _wrap(_ops.dropout_add(self.mlp(h)._t, r, p, self.training))
        return x


def _gpt_attn(layer, h):
    g = getattr(layer, "_rc", None)
    if g == "full_attn":
        from ..distributed.fleet.recompute import recompute
        return recompute(layer.self_attn, h)
    layer.self_attn._rc_core = g == "core_attn"
    return layer.self_attn(h)


class GPTModel(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.config = cfg
        self.embeddings = GPTEmbeddings(cfg)
        self.layers = nn.LayerList([GPTDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.norm = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        if _use_sp(cfg):
            _sp().mark_sequence_parallel(self.norm.weight, self.norm.bias)

    def forward(self, input_ids, position_ids=None):
        if _use_sp(self.config):
            bs = (input_ids.shape[0], input_ids.shape[-1])
            for layer in self.layers:
                layer.self_attn.bs = bs
        x = self.embeddings(input_ids, position_ids)
        rc = self.config.use_recompute and self.training
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
                x = layer(x)
        return self.norm(x)


class GPTForPretraining(nn.Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.config = cfg
        self.gpt = GPTModel(cfg)
        if not cfg.tie_word_embeddings:
            self.lm_head_weight = self.create_parameter([cfg.vocab_size // max(cfg.tensor_parallel_degree, 1),
                                                         cfg.hidden_size],
                                                        default_initializer=I.Normal(0.0, cfg.initializer_range))

    def forward(self, input_ids, position_ids=None, labels=None, loss_mask=None, ignore_index=-100):
        """Logits [B, S, V(_local)]; with ``labels``, the mean token loss instead (through the vocab-sliced
        fused head + CE when config.fused_head_ce and no tensor parallelism, else logits + criterion)."""
        h = self.gpt(input_ids, position_ids)
        w = self.gpt.embeddings.word_embeddings.weight if self.config.tie_word_embeddings else self.lm_head_weight
        ht, wt = h._t, w._t
        if ht.dtype != wt.dtype:
            ht = ht.to(wt.dtype)
        if labels is not None:
            if self.config.fused_head_ce and self.config.tensor_parallel_degree <= 1:
                per_tok = _ops.lm_head_cross_entropy(ht, wt, labels._t, ignore_index)
                return _mean_loss(per_tok, labels._t, loss_mask, ignore_index)
            logits = self.forward(input_ids, position_ids)
            return GPTPretrainingCriterion(self.config, ignore_index)(logits, labels, loss_mask)
        if _use_sp(self.config):
            # token blocks -> vocab-parallel logits of all tokens: the token all-gather overlaps the GEMM of this
            # rank's own block, the backward's dX reduce-scatter overlaps the dW GEMM
            B, S = input_ids.shape[0], input_ids.shape[-1]
            return _wrap(_sp().column_sp_linear_nt(ht, wt).view(B, S, -1))
        if self.config.tensor_parallel_degree > 1:
            ht = _tp().c_identity(ht)
        logits = _ops.linear_nt(ht, wt)  # [B, S, V(_local)]: hand-written GEMM or hipBLASLt per shape
        return _wrap(logits)


class GPTPretrainingCriterion(nn.Layer):
    """Mean token cross-entropy (fused HIP softmax-CE; vocab-parallel CE under TP)."""

    def __init__(self, cfg: GPTConfig = None, ignore_index=-100):
        super().__init__()
        self.cfg = cfg
        self.ignore_index = ignore_index

    def forward(self, logits, labels, loss_mask=None):
        lt = logits._t
        if self.cfg is not None and self.cfg.tensor_parallel_degree > 1:
            per_tok = _tp().parallel_cross_entropy_raw(lt, labels._t, self.ignore_index)
        else:
            per_tok = _ops.softmax_cross_entropy(lt, labels._t, self.ignore_index)
        return _mean_loss(per_tok, labels._t, loss_mask, self.ignore_index)


def _mean_loss(per_tok, labels, loss_mask, ignore_index):
    if loss_mask is not None:
        m = loss_mask._t.reshape(per_tok.shape).float()
        return _wrap((per_tok * m).sum() / m.sum().clamp_min(1.0))
    valid = (labels != ignore_index).sum().clamp_min(1)
    return _wrap(per_tok.sum() / valid)
