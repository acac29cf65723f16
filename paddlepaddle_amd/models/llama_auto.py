"""LLaMA written for semi-automatic parallelism: single-card model code plus placement annotations.

Reference: test/auto_parallel/hybrid_strategy/semi_auto_parallel_llama_model.py (LlamaAttentionAuto,
LlamaMLPAuto, LlamaDecoderLayerAuto, LlamaModelAuto: weights annotated with dist.shard_tensor on the stage
mesh ``global_mesh.get_mesh_with_dim("pp")[ipp]``, column-parallel q/k/v/gate/up (Shard(1) on "mp"),
row-parallel o/down (Shard(0)), hidden states resharded onto the next stage's mesh where a stage starts).

Without a global mesh (``dist.auto_parallel.set_mesh`` not called) it is an ordinary single-card model, which
is how the parallel runs are checked: same seed, same weights, same losses. With a mesh, train it through
``dist.to_static`` (distributed/auto_parallel/static_engine.py): the engine derives tensor / data / pipeline
parallel execution from these annotations.
"""
from __future__ import annotations

import torch

from .. import nn
from .. import ops as _ops
from ..framework.tensor import _wrap
from ..nn import initializer as I
from .llama import LlamaConfig, _Rope

__all__ = ["LlamaForCausalLMAuto", "LlamaPretrainingCriterionAuto", "LlamaConfig"]


def _dist():
    from .. import distributed as dist
    return dist


def _global_mesh():
    return _dist().auto_parallel.get_mesh()


def stage_mesh(ipp):
    gm = _global_mesh()
    if gm is None:
        return None
    if "pp" in gm.dim_names:
        return gm.get_mesh_with_dim("pp", ipp)
    return gm


def num_stages():
    gm = _global_mesh()
    return gm.get_dim_size("pp") if gm is not None and "pp" in gm.dim_names else 1


def _placements(mesh, mp_shard=None, dp_shard=None):
    d = _dist()
    pl = [d.Replicate() for _ in range(mesh.ndim)]
    if mp_shard is not None and "mp" in mesh.dim_names:
        pl[mesh.dim_names.index("mp")] = d.Shard(mp_shard)
    if dp_shard is not None and "dp" in mesh.dim_names:
        pl[mesh.dim_names.index("dp")] = d.Shard(dp_shard)
    return pl


def _shard(layer_param, mesh, mp_shard=None):
    if mesh is None:
        return layer_param
    return _dist().shard_tensor(layer_param, mesh, _placements(mesh, mp_shard))


def _linear(i, o, cfg):
    return nn.Linear(i, o, weight_attr=nn.ParamAttr(initializer=I.Normal(0.0, cfg.initializer_range)), bias_attr=False)


class LlamaRMSNormAuto(nn.Layer):
    def __init__(self, cfg, mesh):
        super().__init__()
        self.weight = self.create_parameter([cfg.hidden_size], default_initializer=I.Constant(1.0))
        _shard(self.weight, mesh)
        self.eps = cfg.rms_norm_eps

    def forward(self, x):
        return _wrap(_ops.rms_norm(x._t, self.weight._t, self.eps))


def _tp_groups(cfg):
    """Tensor-parallel degree the fused projections are laid out for: the global mesh's "mp" size when a mesh is
    set, else cfg.tensor_parallel_degree (dist.parallelize applies the plan after construction)."""
    gm = _global_mesh()
    if gm is not None and "mp" in gm.dim_names:
        return gm.get_dim_size("mp")
    return max(int(getattr(cfg, "tensor_parallel_degree", 1) or 1), 1)


class LlamaAttentionAuto(nn.Layer):
    def __init__(self, cfg, ipp):
        super().__init__()
        self.H, self.Hkv, self.D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        h = cfg.hidden_size
        mesh = stage_mesh(ipp)
        self.fused = bool(getattr(cfg, "fuse_attention_qkv", False))
        if self.fused:
            # [q_r | k_r | v_r] blocks, one per tensor-parallel rank: a column shard is exactly one block
            self.groups = _tp_groups(cfg)
            self.qkv_proj = _linear(h, (self.H + 2 * self.Hkv) * self.D, cfg)
            _shard(self.qkv_proj.weight, mesh, 1)
        else:
            self.q_proj = _linear(h, self.H * self.D, cfg)
            self.k_proj = _linear(h, self.Hkv * self.D, cfg)
            self.v_proj = _linear(h, self.Hkv * self.D, cfg)
            _shard(self.q_proj.weight, mesh, 1)
            _shard(self.k_proj.weight, mesh, 1)
            _shard(self.v_proj.weight, mesh, 1)
        self.o_proj = _linear(self.H * self.D, h, cfg)
        _shard(self.o_proj.weight, mesh, 0)
        self.rope = _Rope(self.D, cfg.rope_theta)

    def forward(self, x):
        B, S = x.shape[0], x.shape[1]
        if self.fused:
            t = self.qkv_proj(x)
            dev = t._t.device
            with torch._C.DisableTorchFunction():
                cos, sin = self.rope.tables(S, torch.device("cpu") if dev.type == "meta" else dev)
                cos, sin = cos[:S], sin[:S]
            o = _ops.qkv_rope_attention(t._t, cos, sin, self.H, self.Hkv, self.D, True, None, True, self.groups)
            return self.o_proj(_wrap(o).reshape([B, S, self.H * self.D]))
        q = self.q_proj(x).reshape([B, S, self.H, self.D])
        k = self.k_proj(x).reshape([B, S, self.Hkv, self.D])
        v = self.v_proj(x).reshape([B, S, self.Hkv, self.D])
        dev = q._t.device
        with torch._C.DisableTorchFunction():  # position tables are constants of a traced program
            cos, sin = self.rope.tables(S, torch.device("cpu") if dev.type == "meta" else dev)
            cos, sin = cos[:S], sin[:S]
        q = _ops.apply_rotary(q._t, cos, sin)
        k = _ops.apply_rotary(k._t, cos, sin)
        o = _ops.flash_attention(q, k, v._t, causal=True)
        return self.o_proj(_wrap(o).reshape([B, S, self.H * self.D]))


class LlamaMLPAuto(nn.Layer):
    def __init__(self, cfg, ipp):
        super().__init__()
        h, f = cfg.hidden_size, cfg.intermediate_size
        mesh = stage_mesh(ipp)
        self.fused = bool(getattr(cfg, "fuse_attention_ffn", False))
        if self.fused:
            # [gate_r | up_r] blocks per tensor-parallel rank; swiglu's one-buffer gradient feeds one dgrad GEMM
            self.groups = _tp_groups(cfg)
            self.f = f
            self.gate_up_proj = _linear(h, 2 * f, cfg)
            _shard(self.gate_up_proj.weight, mesh, 1)
        else:
            self.gate_proj = _linear(h, f, cfg)
            self.up_proj = _linear(h, f, cfg)
            _shard(self.gate_proj.weight, mesh, 1)
            _shard(self.up_proj.weight, mesh, 1)
        self.down_proj = _linear(f, h, cfg)
        _shard(self.down_proj.weight, mesh, 0)

    def forward(self, x):
        if self.fused:
            gu = self.gate_up_proj(x)
            B, S, g = gu.shape[0], gu.shape[1], self.groups
            if g == 1:
                return self.down_proj(_wrap(_ops.swiglu(gu._t)))
            h = _ops.swiglu(gu.reshape([B, S, g, 2 * self.f // g])._t)
            return self.down_proj(_wrap(h).reshape([B, S, self.f]))
        return self.down_proj(_wrap(_ops.swiglu(self.gate_proj(x)._t, self.up_proj(x)._t)))


class LlamaDecoderLayerAuto(nn.Layer):
    def __init__(self, cfg, ipp, stage_start):
        super().__init__()
        self.ipp, self.stage_start = ipp, stage_start
        mesh = stage_mesh(ipp)
        self.input_layernorm = LlamaRMSNormAuto(cfg, mesh)
        self.self_attn = LlamaAttentionAuto(cfg, ipp)
        self.post_attention_layernorm = LlamaRMSNormAuto(cfg, mesh)
        self.mlp = LlamaMLPAuto(cfg, ipp)

    def forward(self, x):
        mesh = stage_mesh(self.ipp)
        if self.stage_start and mesh is not None:
            x = _dist().reshard(x, mesh, _placements(mesh, dp_shard=0))
        h = self.self_attn(self.input_layernorm(x))
        x = x + h
        return x + self.mlp(self.post_attention_layernorm(x))


class LlamaForCausalLMAuto(nn.Layer):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        pp = num_stages()
        L = cfg.num_hidden_layers
        # with virtual_pp_degree v the layers form pp * v chunks, chunk c on pp mesh c % pp (the interleaved layout
        # the static engine's VPP schedule runs: strategy.pipeline.vpp_degree = v, vpp_seg_method =
        # "LlamaDecoderLayerAuto"); v = 1 is the contiguous layout
        nch = pp * max(1, int(getattr(cfg, "virtual_pp_degree", 1) or 1))
        per = max(L // nch, 1)
        first, last = stage_mesh(0), stage_mesh(pp - 1)
        self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size,
                                         weight_attr=nn.ParamAttr(initializer=I.Normal(0.0, cfg.initializer_range)))
        _shard(self.embed_tokens.weight, first)
        self.layers = nn.LayerList([LlamaDecoderLayerAuto(cfg, min(i // per, nch - 1) % pp, i % per == 0 and i > 0)
                                    for i in range(L)])
        self.norm = LlamaRMSNormAuto(cfg, last)
        self.lm_head = _linear(cfg.hidden_size, cfg.vocab_size, cfg)
        _shard(self.lm_head.weight, last, 1)

    def forward(self, input_ids):
        x = self.embed_tokens(input_ids)
        for layer in self.layers:
            x = layer(x)
        return self.lm_head(self.norm(x))


class LlamaPretrainingCriterionAuto(nn.Layer):
    def __init__(self, cfg=None, ignore_index=-100):
        super().__init__()
        self.ignore_index = ignore_index

    def forward(self, logits, labels):
        per_tok = _ops.softmax_cross_entropy(logits._t, labels._t, self.ignore_index)
        valid = (labels._t != self.ignore_index).sum().clamp_min(1)
        return _wrap(per_tok.sum() / valid)
