"""paddlepaddle_amd — a MI355X-native deep-learning framework with PaddlePaddle's ``paddle.*`` API.

Reference API surface: python/paddle/__init__.py (``__all__``, 434 names).
Compute path: PyTorch-ROCm device buffers + hand-written CDNA4 (gfx950) HIP kernels (``ops``),
RCCL over xGMI for collectives (``distributed``), native C++ runtime pieces (``utils.native``).
"""
from __future__ import annotations

import math as _math

import numpy as _np
import torch as _torch

__version__ = "3.0.0+mi355x"

# ---------------------------------------------------------------- core
from .framework import dtype as _dtype_mod
from .framework.dtype import (DType as dtype, uint8, int8, int16, int32, int64, float16, bfloat16,  # noqa: F401
                              float32, float64, complex64, complex128, float8_e4m3fn, float8_e5m2, finfo, iinfo,
                              set_default_dtype, get_default_dtype)
from .framework.dtype import bool_ as bool  # noqa: A001,F401
from .framework.tensor import Tensor, Parameter, to_tensor, is_tensor  # noqa: F401
from .framework.place import (CPUPlace, CUDAPlace, CUDAPinnedPlace, XPUPlace, CustomPlace, IPUPlace,  # noqa: F401
                              set_device, get_device, is_compiled_with_cuda, is_compiled_with_rocm,
                              is_compiled_with_xpu, is_compiled_with_ipu, is_compiled_with_cinn,
                              is_compiled_with_distribute, is_compiled_with_custom_device)
from .framework.grad_mode import no_grad, enable_grad, set_grad_enabled, is_grad_enabled  # noqa: F401
from .framework.random import seed, get_rng_state, set_rng_state, get_cuda_rng_state, set_cuda_rng_state  # noqa: F401
from .framework.flags import set_flags, get_flags  # noqa: F401
from .framework.io import save, load  # noqa: F401
from .framework import in_dynamic_mode, in_dygraph_mode  # noqa: F401

pstring = "pstring"
raw = "raw"

# ---------------------------------------------------------------- ops
from . import tensor  # noqa: F401  (binds Tensor methods)
from .tensor import *  # noqa: F401,F403
from .tensor.creation import range as _range_op  # noqa: F401
from .tensor.einsum import einsum  # noqa: F401
from .tensor import linalg as _linalg_mod
from .tensor.math import inverse  # noqa: F401
from .tensor.linalg import eigvalsh  # noqa: F401
from .tensor.creation import _memcpy  # noqa: F401
from . import ops  # noqa: F401

# ---------------------------------------------------------------- subpackages
from . import autograd, nn, optimizer, amp, io, distributed, device, utils  # noqa: F401
from .autograd import grad, PyLayer  # noqa: F401
from . import linalg, fft, signal, static, jit, metric, vision, hapi, incubate, profiler, distribution, sparse  # noqa: F401,E402
from . import callbacks, text, audio, geometric, quantization, inference, regularizer, onnx, models, parallel  # noqa: F401,E402
import importlib as _il  # noqa: E402
linalg = _il.import_module(".linalg", __name__)  # `from . import linalg` would keep tensor.linalg bound by *
from .hapi import Model, summary, flops  # noqa: F401,E402
from .parallel.data_parallel import DataParallel  # noqa: F401,E402
from .nn.layer.layers import ParamAttr  # noqa: F401,E402
from .static import enable_static, disable_static  # noqa: F401,E402
from .batch import batch  # noqa: F401,E402
from .utils.dlpack import from_dlpack, to_dlpack  # noqa: F401,E402

inf = float("inf")
nan = float("nan")
pi = _math.pi
e = _math.e
newaxis = None


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from .nn.layer.layers import create_parameter_tensor, ParamAttr as _PA
    a = _PA._to_attr(attr)
    if name is not None and a is not False:
        a.name = name
    return create_parameter_tensor(shape, dtype, a, is_bias, default_initializer)


def rank(input):
    return to_tensor(input.ndim, dtype="int32")


def shape(input):
    return to_tensor(input.shape, dtype="int64")


def is_floating_point(x):
    return x._t.is_floating_point()


def is_complex(x):
    return x._t.is_complex()


def is_integer(x):
    return x.is_integer()


def is_empty(x, name=None):
    return to_tensor(x._t.numel() == 0)


def set_printoptions(precision=None, threshold=None, edgeitems=None, sci_mode=None, linewidth=None):
    kw = {k: v for k, v in dict(precision=precision, threshold=threshold, edgeitems=edgeitems,
                                linewidth=linewidth).items() if v is not None}
    _np.set_printoptions(**kw)
    _torch.set_printoptions(**kw)


def check_shape(shape):
    return None


def disable_signal_handler():
    return None


class LazyGuard:
    """Parameters created inside get no memory (meta tensors) until ``param.initialize()`` allocates them on
    their device and runs their initializer (reference: nn/initializer/lazy_init.py) — build a model larger
    than one device, then materialise only the shards a rank keeps."""

    def __enter__(self):
        from .nn.layer import layers as _layers
        _layers._LAZY.depth += 1
        return self

    def __exit__(self, *a):
        from .nn.layer import layers as _layers
        _layers._LAZY.depth -= 1
        return False


def get_cuda_rng_state_list():
    return get_cuda_rng_state()


def tolist(x):
    return x.tolist()


def numel(x, name=None):
    return to_tensor(x._t.numel(), dtype="int64")


def broadcast_shape(x_shape, y_shape):
    return list(_torch.broadcast_shapes(tuple(x_shape), tuple(y_shape)))


def range(start=0, end=None, step=1, dtype=None, name=None):  # noqa: A001
    return arange(start, end, step, dtype)  # noqa: F405


def version_info():
    return __version__


class version:
    full_version = __version__
    major = "3"
    minor = "0"
    patch = "0"
    rc = "0"
    cuda_version = "False"
    cudnn_version = "False"
    hip_version = str(_torch.version.hip)
    istaged = True
    commit = "mi355x"

    @staticmethod
    def show():
        print(f"full_version: {__version__}\nhip: {_torch.version.hip}")

    @staticmethod
    def cuda():
        return "False"

    @staticmethod
    def cudnn():
        return "False"


CUDAPlace = CUDAPlace


def block_diag(inputs, name=None):
    """Block-diagonal matrix from a list of 0-D / 1-D / 2-D tensors (reference tensor/creation.py)."""
    import torch as _t
    from .framework.tensor import _wrap as _w
    ts = []
    for x in inputs:
        t = x._t if hasattr(x, "_t") else _t.as_tensor(x)
        ts.append(t.reshape(1, -1) if t.dim() < 2 else t)
    return _w(_t.block_diag(*ts))


from . import sysconfig, hub, reader, dataset, base, _C_ops, _legacy_C_ops  # noqa: F401,E402
from .tensor import _bind_reference_extras as _bre  # noqa: E402
from .tensor.search import top_p_sampling  # noqa: F401,E402
_bre()


def _maybe_native_allocator():
    """FLAGS_allocator_strategy=auto_growth_best_fit / PADDLE_AMD_ALLOCATOR=auto_growth: install the native
    device allocator (device/allocator.py) before anything touches device memory."""
    from .device import allocator as _al
    if _al._env_requested() and _torch.cuda.is_available():
        _al.enable(int(_os_env.get("PADDLE_AMD_ALLOC_MIN_CHUNK_MB", "64")))


from os import environ as _os_env  # noqa: E402

_maybe_native_allocator()

# reference module paths (paddle.x.y.z files) that this framework implements in an enclosing package
from ._compat_import import install as _install_compat_paths  # noqa: E402
_install_compat_paths()
