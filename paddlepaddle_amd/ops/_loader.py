"""Loader for the hand-written CDNA4 (gfx950) HIP kernel library ``_C_hip.so``.

The library is a plain C-ABI shared object compiled by ``tools/build_native.py`` with
``hipcc --offload-arch=gfx950``. It is loaded with ctypes *after* torch so that it binds to
the HIP runtime instance that torch already loaded (same soname ``libamdhip64.so.7``).

On a machine with a HIP device the kernels are the path that runs; if the library is missing
there we fail loudly (set ``PADDLE_AMD_ALLOW_FALLBACK=1`` to permit the ATen fallback, e.g. for
debugging). On CPU-only hosts the ATen/CPU reference implementations run.
"""
from __future__ import annotations

import ctypes
import os

import torch

from ..framework.flags import flag
from ._sigs import RET_I64, SIGS

_LIB = None
_LIB_ERR = None
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_C_hip.so")


def _load():
    global _LIB, _LIB_ERR
    if _LIB is not None or _LIB_ERR is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        _LIB_ERR = f"{LIB_PATH} not built (run: python tools/build_native.py)"
        return None
    try:
        import torch  # noqa: F401  (bind to torch's HIP runtime first)
        _LIB = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover
        _LIB_ERR = str(e)
        return None
    _declare(_LIB)
    _load_native()
    return _LIB


class _CurrentStream:
    """Sentinel pointer argument: the native launch path substitutes the current HIP stream."""
    __slots__ = ()

    def __repr__(self):
        return "<current HIP stream>"


CURRENT_STREAM = _CurrentStream()
_NATIVE = False   # True once _C_dispatch is loaded: launches skip ctypes
_ENTRY: dict = {}  # launcher name -> METH_FASTCALL entry point of _C_dispatch


def _load_native():
    """Load the generated native entry points (csrc/dispatch). They take tensors, None, ints and the
    CURRENT_STREAM sentinel directly, so ``ptr`` / ``stream_ptr`` hand over the objects unconverted.
    ``PADDLE_AMD_CTYPES_LAUNCH=1`` keeps the ctypes path (A/B timing, debugging)."""
    global _NATIVE
    if os.environ.get("PADDLE_AMD_CTYPES_LAUNCH", "0") == "1":
        return
    try:
        from .. import _C_dispatch as D
    except ImportError:
        return
    D.set_stream_sentinel(CURRENT_STREAM)
    _ENTRY.update({n: getattr(D, n) for n in SIGS if hasattr(D, n)})
    _NATIVE = True


def native_launch() -> bool:
    _load()
    return _NATIVE


def lib():
    l = _load()
    if l is None:
        raise RuntimeError(f"paddlepaddle_amd HIP kernels unavailable: {_LIB_ERR}")
    return l


def hip_enabled_for(t: torch.Tensor) -> bool:
    """True if a HIP kernel should run for a tensor on this device."""
    if not t.is_cuda or not flag("FLAGS_use_hip_kernels", True):
        return False
    if type(t) is not torch.Tensor and type(t) is not torch.nn.Parameter:
        return False  # distributed / wrapper tensors (auto-parallel DTensor) take the sharding-aware path
    if _load() is None:
        if os.environ.get("PADDLE_AMD_ALLOW_FALLBACK", "0") == "1":
            return False
        raise RuntimeError(f"HIP device present but native kernels missing: {_LIB_ERR}")
    return True


def stream_ptr(device=None):
    if _NATIVE and device is None:
        return CURRENT_STREAM
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _declare(L):
    """ctypes argument types of every exported launcher (table in ``_sigs``)."""
    for name, args in SIGS.items():
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = ctypes.c_int64 if name in RET_I64 else ctypes.c_int


def has(name):
    l = _load()
    return l is not None and hasattr(l, name)


# per-launcher dispatch counters: tests assert that the HIP path (not a fallback) ran
CALLS: dict = {}


def calls(name):
    return CALLS.get(name, 0)


def reset_calls():
    CALLS.clear()


def call(name, *args):
    CALLS[name] = CALLS.get(name, 0) + 1
    fn = _ENTRY.get(name)
    rc = fn(*args) if fn is not None else getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"HIP kernel {name} failed with code {rc}")


def ptr(t):
    if _NATIVE:
        return t  # unpacked to data_ptr() in C++
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def dcode(t):
    return _DT[t.dtype]
