"""AMP / numerics debugging. Reference: python/paddle/amp/debugging.py (check_numerics,
enable_operator_stats_collection, TensorCheckerConfig)."""
from __future__ import annotations

import collections
import contextlib

import torch

from ..framework.flags import set_flags
from ..framework.tensor import Tensor, _wrap


class DebugMode:
    CHECK_NAN_INF_AND_ABORT = 0
    CHECK_NAN_INF = 1
    CHECK_ALL_FOR_OVERFLOW = 2
    CHECK_ALL = 3
    CHECK_ALL_AND_ABORT = 4
    DUMP_ALL = 5


def check_numerics(tensor, op_type="", var_name="", debug_mode=DebugMode.CHECK_NAN_INF_AND_ABORT):
    t = tensor._t
    n_nan = int(torch.isnan(t).sum().item()) if t.is_floating_point() else 0
    n_inf = int(torch.isinf(t).sum().item()) if t.is_floating_point() else 0
    if (n_nan or n_inf) and debug_mode in (DebugMode.CHECK_NAN_INF_AND_ABORT, DebugMode.CHECK_ALL_AND_ABORT):
        raise RuntimeError(f"[check_numerics] {op_type}:{var_name} has {n_nan} NaN and {n_inf} Inf values")
    return _wrap(torch.tensor([n_nan, n_inf, 0])), _wrap(torch.tensor([
        float(t.float().max()) if t.numel() else 0.0, float(t.float().min()) if t.numel() else 0.0,
        float(t.float().mean()) if t.numel() else 0.0]))


class TensorCheckerConfig:
    def __init__(self, enable, debug_mode=DebugMode.CHECK_NAN_INF_AND_ABORT, output_dir=None, checked_op_list=None,
                 skipped_op_list=None, debug_step=None, stack_height_limit=1):
        self.enable, self.debug_mode = enable, debug_mode


def enable_tensor_checker(checker_config):
    set_flags({"FLAGS_check_nan_inf": bool(checker_config.enable)})


def disable_tensor_checker():
    set_flags({"FLAGS_check_nan_inf": False})


_op_stats = None


def enable_operator_stats_collection():
    global _op_stats
    _op_stats = collections.Counter()


def disable_operator_stats_collection():
    global _op_stats
    if _op_stats is not None:
        print("<------------------------------------------------------- op list ------------------------------>")
        for k, v in sorted(_op_stats.items()):
            print(f"  {k:<40} | {v}")
    _op_stats = None


@contextlib.contextmanager
def collect_operator_stats():
    enable_operator_stats_collection()
    try:
        yield
    finally:
        disable_operator_stats_collection()


def compare_accuracy(dump_path, another_dump_path, output_filename, loss_scale=1, dump_all_tensors=False):
    raise NotImplementedError("compare_accuracy needs paddle dump files; not produced by this framework")


def check_layer_numerics(func):
    """Decorator for a Layer.forward: checks its tensor inputs and outputs for NaN / Inf
    (reference amp/debugging.py check_layer_numerics)."""
    import functools

    @functools.wraps(func)
    def wrapper(self, *args, **kwargs):
        from ..framework.tensor import Tensor
        name = type(self).__name__
        for i, a in enumerate(args):
            if isinstance(a, Tensor) and a._t.is_floating_point():
                check_numerics(a, name, f"input_{i}", DebugMode.CHECK_NAN_INF_AND_ABORT)
        out = func(self, *args, **kwargs)
        outs = out if isinstance(out, (list, tuple)) else [out]
        for i, o in enumerate(outs):
            if isinstance(o, Tensor) and o._t.is_floating_point():
                check_numerics(o, name, f"output_{i}", DebugMode.CHECK_NAN_INF_AND_ABORT)
        return out
    return wrapper
