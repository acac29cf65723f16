"""Pruning rules of the auto tuner (reference auto_tuner/prune.py): each returns True when the candidate
should be skipped. ``register_prune`` rules see the candidate; ``register_prune_history`` rules also see the
configurations already run (so a config dominated by one that failed is skipped)."""
from __future__ import annotations

from .memory_cost_model import estimate_memory_gb
from .utils import num_gpus

_PRUNE = []
_PRUNE_HISTORY = []


def register_prune(fn):
    _PRUNE.append(fn)
    return fn


def register_prune_history(fn):
    _PRUNE_HISTORY.append(fn)
    return fn


@register_prune
def prune_by_mp(tuner_cfg, cfg, history=()):
    model = tuner_cfg.get("model_cfg", {})
    mp = cfg["mp_degree"]
    for k in ("hidden_size", "num_attention_heads", "vocab_size"):
        if model.get(k) and model[k] % mp:
            return True
    return mp > int(tuner_cfg.get("gpus_per_node", 8))  # TP stays inside one node's xGMI ring


@register_prune
def prune_by_pp(tuner_cfg, cfg, history=()):
    layers = tuner_cfg.get("model_cfg", {}).get("num_layers")
    pp = cfg["pp_degree"]
    if layers and layers % pp:
        return True
    return pp > 1 and cfg.get("acc_steps", 1) < pp  # fewer micro-batches than stages: bubble dominates


@register_prune
def prune_by_sharding(tuner_cfg, cfg, history=()):
    return cfg["sharding_degree"] == 1 and cfg["sharding_stage"] != 1  # stages only differ with a group


@register_prune
def prune_by_num_gpus(tuner_cfg, cfg, history=()):
    return cfg["dp_degree"] * cfg["mp_degree"] * cfg["pp_degree"] != num_gpus(tuner_cfg)


@register_prune
def prune_by_memory_estimation(tuner_cfg, cfg, history=()):
    model = tuner_cfg.get("model_cfg")
    if not model or "hidden_size" not in model or "num_layers" not in model:
        return False
    limit = float(tuner_cfg.get("max_mem_usage", 288 * 0.9))
    cfg["estimated_memory_gb"] = round(estimate_memory_gb(cfg, model), 2)
    return cfg["estimated_memory_gb"] > limit


@register_prune_history
def prune_by_oom_history(tuner_cfg, cfg, history=()):
    """A config that keeps everything of an out-of-memory run but a larger micro-batch, or no recompute where
    that run recomputed, needs at least as much memory: skip it."""
    for h in history:
        if not h.get("oom"):
            continue
        same = all(h.get(k) == cfg.get(k) for k in ("dp_degree", "mp_degree", "pp_degree", "sharding_degree",
                                                      "sharding_stage", "vpp_degree"))
        if not same:
            continue
        if cfg["micro_batch_size"] >= h["micro_batch_size"] and (not cfg["use_recompute"] or h["use_recompute"]):
            return True
    return False


def prune(tuner_cfg, cfg, history=()):
    if any(fn(tuner_cfg, cfg, history) for fn in _PRUNE):
        return True
    return any(fn(tuner_cfg, cfg, history) for fn in _PRUNE_HISTORY)
