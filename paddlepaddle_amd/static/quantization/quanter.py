"""Static-graph quantization-aware training. Reference: python/paddle/static/quantization/quanter.py (quant_aware,
convert; the PaddleSlim config dict).

quant_aware inserts, ahead of every quantizable op (conv2d / mul / matmul with a constant weight), an
activation fake-quant node (moving-average abs-max scale in a program buffer, straight-through gradient) and a
weight fake-quant node (channel-wise or per-tensor abs max); the program keeps training through them.
convert replaces the activation nodes by fixed-scale quant-dequant nodes and folds the weight quantisation
into the weights, ready for save_inference_model."""
from __future__ import annotations

import copy

import torch

from .. import program as P
from . import _graph as G
from . import quant_ops as Q

_DEFAULT = {
    "weight_quantize_type": "channel_wise_abs_max",
    "activation_quantize_type": "moving_average_abs_max",
    "weight_bits": 8,
    "activation_bits": 8,
    "not_quant_pattern": ["skip_quant"],
    "quantize_op_types": ["conv2d", "depthwise_conv2d", "mul"],
    "dtype": "int8",
    "window_size": 10000,
    "moving_rate": 0.9,
    "for_tensorrt": False,
    "is_full_quantize": False,
    "onnx_format": False,
}


def _config(config):
    cfg = dict(_DEFAULT)
    cfg.update(config or {})
    if cfg["weight_quantize_type"] not in ("abs_max", "channel_wise_abs_max"):
        raise ValueError(f"unsupported weight_quantize_type {cfg['weight_quantize_type']}")
    if cfg["activation_quantize_type"] not in ("moving_average_abs_max", "abs_max", "range_abs_max"):
        raise ValueError(f"unsupported activation_quantize_type {cfg['activation_quantize_type']}")
    return cfg


def quant_aware(program, place=None, config=None, scope=None, for_test=False, weight_quantize_func=None,
                act_quantize_func=None, weight_preprocess_func=None, act_preprocess_func=None,
                optimizer_func=None, executor=None, return_program=True, draw_graph=False):
    cfg = _config(config)
    prog = program.clone(for_test=for_test) if for_test else program
    types = set(cfg["quantize_op_types"]) | ({"matmul", "mul"} if cfg["is_full_quantize"] else set())
    rate = cfg["moving_rate"] if cfg["activation_quantize_type"] == "moving_average_abs_max" else 0.0
    nodes = G.quantizable_nodes(prog, types)
    prog._quant_nodes = []
    for _, node, ref_type, w, axis in nodes:
        with G.raw():
            state = torch.zeros(2, dtype=torch.float32, device=w.t.device)   # [scale, steps]
        act = G.insert_before(prog, node, Q.qat_fake_quant_act,
                              (prog._const(state), rate, cfg["activation_bits"]), 0)
        waxis = axis if cfg["weight_quantize_type"] == "channel_wise_abs_max" else None
        wq = G.insert_before(prog, node, Q.qat_fake_quant_weight, (waxis, cfg["weight_bits"]), 1)
        prog._quant_nodes.append((node, act, wq, state, w, waxis))
    prog._quant_config = cfg
    return prog


def convert(program, place=None, config=None, scope=None, save_int8=False):
    """Freeze a quant_aware program: fixed activation scales, weights replaced by their quantised values."""
    cfg = _config(config or getattr(program, "_quant_config", None))
    prog = program.clone(for_test=True) if hasattr(program, "clone") else copy.copy(program)
    src = getattr(program, "_quant_nodes", [])
    by_id = {id(n): n for n in program.nodes}
    idx_of = {id(n): i for i, n in enumerate(program.nodes)}
    for node, act, wq, state, w, waxis in src:
        if id(act) not in by_id:
            continue
        a = prog.nodes[idx_of[id(act)]]
        a.func, a.name = Q.fake_quant_act, P._func_name(Q.fake_quant_act)
        with G.raw():
            a.args = (a.args[0], float(state[0]), int(cfg["activation_bits"]))
        with torch.no_grad(), G.raw():
            w.t.copy_(Q.qat_fake_quant_weight(w.t.detach(), waxis, cfg["weight_bits"]))
        q = prog.nodes[idx_of[id(wq)]]
        # the weight node becomes an identity on the (already quantised) constant
        q.func, q.name = torch.clone, P._func_name(torch.clone)
        q.args = (q.args[0],)
    prog._version += 1
    prog._plans.clear()
    return prog
