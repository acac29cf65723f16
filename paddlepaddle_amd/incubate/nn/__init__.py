"""paddle.incubate.nn: fused layers. Reference: python/paddle/incubate/nn/layer/fused_*.py."""
from __future__ import annotations

from ... import nn as _nn
from ...nn import initializer as _I
from . import functional  # noqa: F401
from . import functional as F


class FusedLinear(_nn.Layer):
    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, transpose_weight=False,
                 name=None):
        super().__init__()
        shape = [out_features, in_features] if transpose_weight else [in_features, out_features]
        self.weight = self.create_parameter(shape, attr=weight_attr)
        self.bias = self.create_parameter([out_features], attr=bias_attr, is_bias=True) if bias_attr is not False \
            else None
        self.transpose_weight = transpose_weight

    def forward(self, x):
        return F.fused_linear(x, self.weight, self.bias, self.transpose_weight)


class FusedDropoutAdd(_nn.Layer):
    def __init__(self, p=0.5, mode="upscale_in_train", name=None):
        super().__init__()
        self.p, self.mode = p, mode

    def forward(self, x, y):
        return F.fused_dropout_add(x, y, self.p, self.training, self.mode)


class FusedBiasDropoutResidualLayerNorm(_nn.Layer):
    def __init__(self, embed_dim, dropout_rate=0.5, weight_attr=None, bias_attr=None, epsilon=1e-5, name=None):
        super().__init__()
        self.linear_bias = self.create_parameter([embed_dim], attr=bias_attr, is_bias=True)
        self.ln_scale = self.create_parameter([embed_dim], attr=weight_attr, default_initializer=_I.Constant(1.0))
        self.ln_bias = self.create_parameter([embed_dim], is_bias=True)
        self.dropout_rate, self.epsilon = dropout_rate, epsilon

    def forward(self, x, residual):
        return F.fused_bias_dropout_residual_layer_norm(x, residual, self.linear_bias, self.ln_scale, self.ln_bias,
                                                        self.dropout_rate, self.epsilon, self.training)


class FusedFeedForward(_nn.Layer):
    def __init__(self, d_model, dim_feedforward, dropout_rate=0.1, epsilon=1e-05, activation="relu",
                 act_dropout_rate=None, normalize_before=False, linear1_weight_attr=None, linear1_bias_attr=None,
                 linear2_weight_attr=None, linear2_bias_attr=None, ln1_scale_attr=None, ln1_bias_attr=None,
                 ln2_scale_attr=None, ln2_bias_attr=None, nranks=1, ring_id=-1, name=None):
        super().__init__()
        self._d = d_model
        self.normalize_before = normalize_before
        self.dropout_rate = dropout_rate
        self.act_dropout_rate = dropout_rate if act_dropout_rate is None else act_dropout_rate
        self.activation = activation
        self.epsilon = epsilon
        self._linear1_weight = self.create_parameter([d_model, dim_feedforward], attr=linear1_weight_attr)
        self._linear1_bias = self.create_parameter([dim_feedforward], attr=linear1_bias_attr, is_bias=True)
        self._linear2_weight = self.create_parameter([dim_feedforward, d_model], attr=linear2_weight_attr)
        self._linear2_bias = self.create_parameter([d_model], attr=linear2_bias_attr, is_bias=True)
        one = _I.Constant(1.0)
        self._ln1_scale = self.create_parameter([d_model], attr=ln1_scale_attr, default_initializer=one)
        self._ln1_bias = self.create_parameter([d_model], attr=ln1_bias_attr, is_bias=True)
        self._ln2_scale = self.create_parameter([d_model], attr=ln2_scale_attr, default_initializer=one)
        self._ln2_bias = self.create_parameter([d_model], attr=ln2_bias_attr, is_bias=True)

    def forward(self, src, cache=None):
        return F.fused_feedforward(src, self._linear1_weight, self._linear2_weight, self._linear1_bias,
                                   self._linear2_bias, self._ln1_scale, self._ln1_bias, self._ln2_scale,
                                   self._ln2_bias, self.act_dropout_rate, self.dropout_rate, self.activation,
                                   self.epsilon, self.epsilon, self.normalize_before, self.training)


class FusedMultiHeadAttention(_nn.Layer):
    def __init__(self, embed_dim, num_heads, dropout_rate=0.5, attn_dropout_rate=0.5, kdim=None, vdim=None,
                 normalize_before=False, need_weights=False, qkv_weight_attr=None, qkv_bias_attr=None,
                 linear_weight_attr=None, linear_bias_attr=None, pre_ln_scale_attr=None, pre_ln_bias_attr=None,
                 ln_scale_attr=None, ln_bias_attr=None, epsilon=1e-5, nranks=1, ring_id=-1, transpose_qkv_wb=False,
                 name=None):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.normalize_before = normalize_before
        self.dropout_rate, self.attn_dropout_rate = dropout_rate, attn_dropout_rate
        self.epsilon = epsilon
        self.transpose_qkv_wb = transpose_qkv_wb
        qshape = [embed_dim, 3 * embed_dim] if transpose_qkv_wb else [3, num_heads, self.head_dim, embed_dim]
        self.qkv_weight = self.create_parameter(qshape, attr=qkv_weight_attr)
        self.qkv_bias = self.create_parameter([3 * embed_dim] if transpose_qkv_wb else [3, num_heads, self.head_dim],
                                              attr=qkv_bias_attr, is_bias=True)
        self.linear_weight = self.create_parameter([embed_dim, embed_dim], attr=linear_weight_attr)
        self.linear_bias = self.create_parameter([embed_dim], attr=linear_bias_attr, is_bias=True)
        one = _I.Constant(1.0)
        self.pre_ln_scale = self.create_parameter([embed_dim], attr=pre_ln_scale_attr, default_initializer=one)
        self.pre_ln_bias = self.create_parameter([embed_dim], attr=pre_ln_bias_attr, is_bias=True)
        self.ln_scale = self.create_parameter([embed_dim], attr=ln_scale_attr, default_initializer=one)
        self.ln_bias = self.create_parameter([embed_dim], attr=ln_bias_attr, is_bias=True)

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        return F.fused_multi_head_attention(query, self.qkv_weight, self.linear_weight, self.normalize_before,
                                            self.pre_ln_scale, self.pre_ln_bias, self.ln_scale, self.ln_bias,
                                            self.epsilon, self.qkv_bias, self.linear_bias, None, attn_mask,
                                            self.dropout_rate, self.attn_dropout_rate, self.epsilon, self.training,
                                            num_heads=self.num_heads, transpose_qkv_wb=self.transpose_qkv_wb)


class FusedTransformerEncoderLayer(_nn.Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout_rate=0.1, activation="relu", attn_dropout_rate=None,
                 act_dropout_rate=None, normalize_before=False, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self.fused_attn = FusedMultiHeadAttention(d_model, nhead, dropout_rate,
                                                  dropout_rate if attn_dropout_rate is None else attn_dropout_rate,
                                                  normalize_before=normalize_before)
        self.ffn = FusedFeedForward(d_model, dim_feedforward, dropout_rate, activation=activation,
                                    act_dropout_rate=act_dropout_rate, normalize_before=normalize_before)

    def forward(self, src, src_mask=None, cache=None):
        return self.ffn(self.fused_attn(src, attn_mask=src_mask))


class FusedMultiTransformer(_nn.Layer):
    """Stack of generation decoder layers over F.fused_multi_transformer (reference
    incubate/nn/layer/fused_transformer.py FusedMultiTransformer): per-layer parameter lists, qkv weight
    [3, H, D, E] (or [E, 3, H, D] without trans_qkvw; [H + 2*kv, D, E] with gqa_group_size = kv heads),
    heads / ffn width split over nranks tensor-parallel ranks (ring_id selects the mp all-reduce)."""

    def __init__(self, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0, activation="gelu",
                 normalize_before=True, ln_scale_attrs=None, ln_bias_attrs=None, qkv_weight_attrs=None,
                 qkv_bias_attrs=None, linear_weight_attrs=None, linear_bias_attrs=None, ffn_ln_scale_attrs=None,
                 ffn_ln_bias_attrs=None, ffn1_weight_attrs=None, ffn1_bias_attrs=None, ffn2_weight_attrs=None,
                 ffn2_bias_attrs=None, epsilon=1e-5, residual_alpha=1.0, num_layers=-1, nranks=1, trans_qkvw=True,
                 ring_id=-1, norm_type="layernorm", use_neox_rotary_style=False, gqa_group_size=-1, name=None):
        super().__init__()
        if embed_dim <= 0 or num_heads <= 0 or dim_feedforward <= 0:
            raise ValueError("embed_dim, num_heads and dim_feedforward must be positive")
        if num_heads % nranks or dim_feedforward % nranks:
            raise ValueError("num_heads and dim_feedforward must divide by nranks")
        if num_layers < 0:
            num_layers = len(qkv_weight_attrs) if isinstance(qkv_weight_attrs, (list, tuple)) else 1
        self.normalize_before, self.dropout_rate, self.activation = normalize_before, dropout_rate, activation
        self._epsilon, self._residual_alpha, self._trans_qkvw = epsilon, residual_alpha, trans_qkvw
        self._ring_id, self._norm_type = ring_id, norm_type
        self._use_neox_rotary_style, self._gqa_group_size = use_neox_rotary_style, gqa_group_size
        self.head_dim = embed_dim // num_heads
        H = num_heads // nranks
        kv = (gqa_group_size // nranks) if gqa_group_size and gqa_group_size > 0 else None
        ffn = dim_feedforward // nranks
        heads_shape = [3, H] if kv is None else [H + 2 * kv]

        def attr(a, i):
            return a[i] if isinstance(a, (list, tuple)) else a

        names = ["ln_scales", "ln_biases", "qkv_weights", "qkv_biases", "linear_weights", "linear_biases",
                 "ffn_ln_scales", "ffn_ln_biases", "ffn1_weights", "ffn1_biases", "ffn2_weights", "ffn2_biases"]
        for n in names:
            setattr(self, n, _nn.ParameterList())
        one, zero = _I.Constant(1.0), _I.Constant(0.0)
        for i in range(num_layers):
            self.ln_scales.append(self.create_parameter([embed_dim], attr=attr(ln_scale_attrs, i),
                                                        default_initializer=one))
            self.ln_biases.append(self.create_parameter([embed_dim], attr=attr(ln_bias_attrs, i), is_bias=True))
            qkv_shape = ([*heads_shape, self.head_dim, embed_dim] if trans_qkvw
                         else [embed_dim, *heads_shape, self.head_dim])
            self.qkv_weights.append(self.create_parameter(qkv_shape, attr=attr(qkv_weight_attrs, i)))
            self.qkv_biases.append(self.create_parameter([*heads_shape, self.head_dim],
                                                         attr=attr(qkv_bias_attrs, i), is_bias=True))
            self.linear_weights.append(self.create_parameter([H * self.head_dim, embed_dim],
                                                             attr=attr(linear_weight_attrs, i)))
            self.linear_biases.append(self.create_parameter([embed_dim], attr=attr(linear_bias_attrs, i),
                                                            is_bias=True))
            self.ffn_ln_scales.append(self.create_parameter([embed_dim], attr=attr(ffn_ln_scale_attrs, i),
                                                            default_initializer=one))
            self.ffn_ln_biases.append(self.create_parameter([embed_dim], attr=attr(ffn_ln_bias_attrs, i),
                                                            is_bias=True))
            self.ffn1_weights.append(self.create_parameter([embed_dim, ffn], attr=attr(ffn1_weight_attrs, i)))
            self.ffn1_biases.append(self.create_parameter([ffn], attr=attr(ffn1_bias_attrs, i), is_bias=True))
            self.ffn2_weights.append(self.create_parameter([ffn, embed_dim], attr=attr(ffn2_weight_attrs, i)))
            self.ffn2_biases.append(self.create_parameter([embed_dim], attr=attr(ffn2_bias_attrs, i), is_bias=True))
        del zero

    def forward(self, src, attn_mask=None, caches=None, pre_caches=None, rotary_embs=None, rotary_emb_dims=0,
                beam_offset=None, seq_lens=None, time_step=None):
        return F.fused_multi_transformer(
            src, list(self.ln_scales), list(self.ln_biases), list(self.qkv_weights), list(self.qkv_biases),
            list(self.linear_weights), list(self.linear_biases), list(self.ffn_ln_scales),
            list(self.ffn_ln_biases), list(self.ffn1_weights), list(self.ffn1_biases), list(self.ffn2_weights),
            list(self.ffn2_biases), pre_layer_norm=self.normalize_before, epsilon=self._epsilon,
            residual_alpha=self._residual_alpha, cache_kvs=caches, beam_offset=beam_offset, pre_caches=pre_caches,
            seq_lens=seq_lens, rotary_embs=rotary_embs, time_step=time_step, attn_mask=attn_mask,
            dropout_rate=self.dropout_rate, rotary_emb_dims=rotary_emb_dims, activation=self.activation,
            training=self.training, trans_qkvw=self._trans_qkvw, ring_id=self._ring_id, norm_type=self._norm_type,
            use_neox_rotary_style=self._use_neox_rotary_style, gqa_group_size=self._gqa_group_size)
