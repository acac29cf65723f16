"""Candidate generation and trial-argument plumbing of the auto tuner (reference auto_tuner/utils.py)."""
from __future__ import annotations

import itertools
import re

KEYS = ("dp_degree", "mp_degree", "pp_degree", "vpp_degree", "sharding_degree", "sharding_stage",
        "micro_batch_size", "use_recompute")


def divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


def num_gpus(tuner_cfg):
    if "num_gpus" in tuner_cfg:
        return int(tuner_cfg["num_gpus"])
    return int(tuner_cfg.get("nodes", 1)) * int(tuner_cfg.get("gpus_per_node", 8))


def _cands(value, auto):
    if value is None or value == "auto":
        return list(auto)
    return list(value) if isinstance(value, (list, tuple)) else [value]


def default_candidates(tuner_cfg):
    """Per-dimension candidate lists; "auto" (or absent) expands to every value that can divide the job."""
    n = num_gpus(tuner_cfg)
    model = tuner_cfg.get("model_cfg", {})
    gpn = int(tuner_cfg.get("gpus_per_node", min(n, 8)))
    layers = int(model.get("num_layers", 1))
    gbs = int(model.get("global_batch_size", 1))
    heads = model.get("num_attention_heads")
    mp_auto = [d for d in divisors(n) if d <= gpn and (heads is None or heads % d == 0)]
    pp_auto = [d for d in divisors(n) if layers % d == 0]
    c = {
        "dp_degree": _cands(tuner_cfg.get("dp_degree"), divisors(n)),
        "mp_degree": _cands(tuner_cfg.get("mp_degree"), mp_auto),
        "pp_degree": _cands(tuner_cfg.get("pp_degree"), pp_auto),
        "vpp_degree": _cands(tuner_cfg.get("vpp_degree"), [1]),
        "sharding_degree": _cands(tuner_cfg.get("sharding_degree"), divisors(n)),
        "sharding_stage": _cands(tuner_cfg.get("sharding_stage"), [1, 2, 3]),
        "micro_batch_size": _cands(tuner_cfg.get("micro_batch_size"), divisors(gbs)),
        "use_recompute": _cands(tuner_cfg.get("use_recompute"), [False, True]),
    }
    return c


def search_all(tuner_cfg):
    """Every combination of the candidates whose degrees tile the GPUs and whose batch splits evenly:
    dp * mp * pp = #GPUs, sharding_degree divides dp (the sharding group lives inside the data-parallel
    ranks), gbs % (dp * mbs) == 0, layers % (pp * vpp) == 0."""
    c = tuner_cfg.get("candidates") or default_candidates(tuner_cfg)
    n = num_gpus(tuner_cfg)
    model = tuner_cfg.get("model_cfg", {})
    gbs = int(model.get("global_batch_size", 1))
    layers = int(model.get("num_layers", 1))
    out = []
    for combo in itertools.product(*(c[k] for k in KEYS)):
        cfg = dict(zip(KEYS, combo))
        dp, mp, pp, vpp = cfg["dp_degree"], cfg["mp_degree"], cfg["pp_degree"], cfg["vpp_degree"]
        if dp * mp * pp != n or dp % cfg["sharding_degree"]:
            continue
        if gbs % (dp * cfg["micro_batch_size"]) or layers % (pp * vpp):
            continue
        if vpp > 1 and pp == 1:
            continue
        cfg["acc_steps"] = gbs // (dp * cfg["micro_batch_size"])
        out.append(cfg)
    return out


def gen_new_args(raw_args, cfg, tuner_cfg):
    """The trial's script arguments: ``tuner_cfg["run_cmd"]`` maps a config key to a flag template,
    e.g. {"mp_degree": ["--tp", "{value}"], "use_recompute": ["--recompute", "{value:d}"]}; a flag that is
    already in the arguments gets its value replaced, otherwise it is appended."""
    args = list(raw_args)
    for key, tmpl in (tuner_cfg.get("run_cmd") or {}).items():
        if key not in cfg:
            continue
        flag, vt = tmpl[0], tmpl[1] if len(tmpl) > 1 else "{value}"
        v = cfg[key]
        value = vt.format(value=int(v) if isinstance(v, bool) else v)
        if flag in args:
            i = args.index(flag)
            if i + 1 < len(args):
                args[i + 1] = value
            else:
                args.append(value)
        else:
            args += [flag, value]
    return args


def parse_metric(text, metric_cfg):
    """Last value of the metric in a worker log: ``metric_cfg["regex"]`` (one group) or
    '<name>' followed by '=' / ':' and a number."""
    pat = metric_cfg.get("regex") or (re.escape(metric_cfg["name"]) + r"\s*[=:]\s*([0-9.eE+-]+)")
    vals = re.findall(pat, text)
    if not vals:
        return None
    try:
        return float(vals[-1])
    except ValueError:
        return None
