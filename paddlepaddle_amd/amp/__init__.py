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


class AMPGlobalState:
    """What decorate() recorded for the rest of the run (reference auto_cast.py AMPGlobalState): the decorated
    models' parameters, whether gradients of low-precision parameters are kept in fp32 (master_grad) and the
    low-precision dtype."""

    def __init__(self):
        self.model_parameters = []
        self.use_master_grad = False
        self.already_register_final_backward_hook = False
        self.already_classify_params_meets_need = False
        self.amp_dtype = "float32"

    def __setattr__(self, name, value):
        self.__dict__[name] = value


_AMP_GLOBAL = AMPGlobalState()


def amp_global_state():
    return _AMP_GLOBAL


def amp_state():
    """The auto_cast state in force (enabled, level, dtype, op lists)."""
    return STATE


def _norm_types():
    from ..nn.layer.norm import _BatchNormBase, LayerNorm, GroupNorm, _InstanceNormBase
    return (_BatchNormBase, LayerNorm, GroupNorm, _InstanceNormBase)


def need_keep_fp32(layer, dtype):
    """O2 keeps normalization layers (and layers marked by set_excluded_layers) in fp32."""
    return isinstance(layer, _norm_types()) or getattr(layer, "_cast_to_low_precision", True) is False


def set_excluded_layers(models, excluded_layers):
    """Mark layers (instances, or every sublayer of the given types) to stay fp32 under O2 decorate."""
    ms = models if isinstance(models, (list, tuple)) else [models]
    ex = excluded_layers if isinstance(excluded_layers, (list, tuple)) else [excluded_layers]
    types_ = tuple(e for e in ex if isinstance(e, type))
    insts = [e for e in ex if not isinstance(e, type)]
    for m in ms:
        for l in m.sublayers(include_self=True):
            if (types_ and isinstance(l, types_)) or any(l is i for i in insts):
                for sub in l.sublayers(include_self=True):
                    object.__setattr__(sub, "_cast_to_low_precision", False)


def check_models(models):
    from ..nn.layer.layers import Layer
    for m in models:
        if not isinstance(m, Layer):
            raise RuntimeError(f"Current train mode is pure fp16, models should be paddle.nn.Layer, but receive "
                               f"{type(m)}.")


def check_optimizers(optimizers):
    from ..optimizer.optimizer import Optimizer
    for o in optimizers:
        if not isinstance(o, Optimizer):
            raise RuntimeError(f"Current train mode is pure fp16, optimizers should be paddle.optimizer.Optimizer,"
                               f" but receive {type(o)}.")


def decorate(models, optimizers=None, level="O1", dtype="float16", master_weight=None, save_dtype=None,
             master_grad=False, excluded_layers=None):
    """O2: cast model parameters to dtype (norm layers stay fp32) and turn on optimizer master weights."""
    single_model = not isinstance(models, (list, tuple))
    ms = [models] if single_model else list(models)
    if level == "O2":
        check_models(ms)
        td = _dt.to_torch_dtype(dtype)
        if excluded_layers is not None:
            set_excluded_layers(ms, excluded_layers)
        g = amp_global_state()
        g.use_master_grad = bool(master_grad)
        g.amp_dtype = dtype
        for m in ms:
            g.model_parameters.extend(m.parameters())
            for l in m.sublayers(include_self=True):
                if need_keep_fp32(l, dtype):
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


amp_decorate = decorate


def is_auto_cast_enabled():
    return STATE.enabled


def get_amp_dtype():
    return _dt.from_torch_dtype(STATE.dtype).name if STATE.enabled else "float32"
