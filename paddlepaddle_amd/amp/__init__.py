"""paddle.amp. Reference: python/paddle/amp/{auto_cast.py:1029 auto_cast, :1114 decorate,
grad_scaler.py:657 GradScaler}."""
from __future__ import annotations

import contextlib

import torch

from ..framework import dtype as _dt
from ..framework.tensor import Tensor, _wrap
from . import debugging  # noqa: F401
from .state import STATE, WHITE_LIST, BLACK_LIST
from .grad_scaler import GradScaler, AmpScaler, OptimizerState  # noqa: F401


def is_float16_supported(device=None):
    return True


def is_bfloat16_supported(device=None):
    return True


@contextlib.contextmanager
def auto_cast(enable=True, custom_white_list=None, custom_black_list=None, level="O1", dtype="float16",
              use_promote=True):
    prev = (STATE.enabled, STATE.level, STATE.dtype, set(STATE.white), set(STATE.black))
    try:
        if enable and level in ("O1", "O2"):
            STATE.enabled = True
            STATE.level = level
            STATE.dtype = _dt.to_torch_dtype(dtype)
            if custom_white_list:
                STATE.white |= set(custom_white_list)
                STATE.black -= set(custom_white_list)
            if custom_black_list:
                STATE.black |= set(custom_black_list)
                STATE.white -= set(custom_black_list)
        else:
            STATE.enabled = False
        yield
    finally:
        STATE.enabled, STATE.level, STATE.dtype, STATE.white, STATE.black = prev


amp_guard = auto_cast


def decorate(models, optimizers=None, level="O1", dtype="float16", master_weight=None, save_dtype=None,
             master_grad=False, excluded_layers=None):
    """O2: cast model parameters to dtype (norm layers stay fp32) and turn on optimizer master weights."""
    from ..nn.layer.norm import _BatchNormBase, LayerNorm, GroupNorm, _InstanceNormBase
    single_model = not isinstance(models, (list, tuple))
    ms = [models] if single_model else list(models)
    if level == "O2":
        td = _dt.to_torch_dtype(dtype)
        keep = (_BatchNormBase, LayerNorm, GroupNorm, _InstanceNormBase)
        if excluded_layers is not None:
            ex = excluded_layers if isinstance(excluded_layers, (list, tuple)) else [excluded_layers]
            keep = keep + tuple(e for e in ex if isinstance(e, type))
        for m in ms:
            for l in m.sublayers(include_self=True):
                if isinstance(l, keep):
                    continue
                for p in l._parameters.values():
                    if p is not None and p._t.is_floating_point() and p._t.dtype != td:
                        p._replace_data(p._t.to(td))
            m._casted_by_pure_fp16 = True
        if optimizers is not None:
            os_ = optimizers if isinstance(optimizers, (list, tuple)) else [optimizers]
            for o in os_:
                if master_weight is None or master_weight:
                    o._multi_precision = True
    if optimizers is None:
        return models
    return models, optimizers


def is_auto_cast_enabled():
    return STATE.enabled


def get_amp_dtype():
    return _dt.from_torch_dtype(STATE.dtype).name if STATE.enabled else "float32"
