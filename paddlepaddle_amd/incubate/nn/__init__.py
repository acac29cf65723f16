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
    def __init__(self, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0, activation="gelu",
                 normalize_before=True, num_layers=1, epsilon=1e-5, name=None, **kw):
        super().__init__()
        self.layers = _nn.LayerList([FusedTransformerEncoderLayer(embed_dim, num_heads, dim_feedforward,
                                                                  dropout_rate, activation,
                                                                  normalize_before=normalize_before)
                                     for _ in range(num_layers)])

    def forward(self, src, attn_mask=None, caches=None, time_step=None, **kw):
        h = src
        for l in self.layers:
            h = l(h, attn_mask)
        return h
