"""Per-GPU memory of a decoder-only LM training step under a hybrid-parallel configuration
(reference auto_tuner/memory_cost_model.py). bf16 weights / grads, fp32 master weights + Adam moments
(12 bytes per parameter) sharded by the sharding stage, activations after Korthikanti et al.
(s * b * h * (34 + 5 a s / h) bytes per layer, / mp with sequence parallelism; 2 s b h with full
recompute), 1F1B keeping up to pp micro-batches of activations in flight on the first stage."""
from __future__ import annotations


def estimate_memory_gb(cfg, model_cfg):
    h = int(model_cfg["hidden_size"])
    L = int(model_cfg["num_layers"])
    V = int(model_cfg.get("vocab_size", 50304))
    s = int(model_cfg.get("seq_length", 2048))
    a = int(model_cfg.get("num_attention_heads", max(h // 128, 1)))
    ffn = int(model_cfg.get("intermediate_size", 4 * h))
    mp, pp = cfg["mp_degree"], cfg["pp_degree"]
    sd, stage = cfg.get("sharding_degree", 1), cfg.get("sharding_stage", 1)
    b = cfg["micro_batch_size"]
    per_layer = 4 * h * h + 2 * h * ffn + 4 * h
    params = (L * per_layer / pp + V * h) / mp
    weights = 2 * params / (sd if stage >= 3 else 1)
    grads = 2 * params / (sd if stage >= 2 else 1)
    opt = 12 * params / sd
    layers_here = L / pp
    if cfg.get("use_recompute"):
        act_layer = 2 * s * b * h
    else:
        act_layer = s * b * h * (34 + 5 * a * s / h) / mp
    in_flight = min(pp, cfg.get("acc_steps", pp))
    act = act_layer * layers_here * in_flight
    logits = 4 * s * b * V / mp  # bf16 logits + their gradient on the last stage
    return (weights + grads + opt + act + logits) / 1e9
