"""paddle.utils. Reference: python/paddle/utils/."""
from __future__ import annotations

import functools
import itertools
import warnings

from . import native  # noqa: F401
from . import unique_name  # noqa: F401
from . import dlpack  # noqa: F401
from . import cpp_extension  # noqa: F401


def deprecated(update_to="", since="", reason="", level=0):
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **k):
            warnings.warn(f"{fn.__name__} is deprecated since {since}: {reason} {update_to}", DeprecationWarning)
            return fn(*a, **k)
        return wrapper
    return deco


def run_check():
    """paddle.utils.run_check: build + run a tiny model on the available device."""
    import paddlepaddle_amd as paddle
    x = paddle.randn([4, 8])
    lin = paddle.nn.Linear(8, 2)
    y = lin(x).sum()
    y.backward()
    dev = paddle.get_device()
    print(f"PaddlePaddle-AMD works well on {dev}. HIP kernels: {paddle.ops.has_kernel('pa_version')}")


def try_import(module_name, err_msg=None):
    import importlib
    try:
        return importlib.import_module(module_name)
    except ImportError:
        raise ImportError(err_msg or f"{module_name} is required")


def flatten(nest):
    out = []
    if isinstance(nest, (list, tuple)):
        for n in nest:
            out.extend(flatten(n))
    elif isinstance(nest, dict):
        for k in sorted(nest):
            out.extend(flatten(nest[k]))
    else:
        out.append(nest)
    return out


def map_structure(func, *structure):
    s0 = structure[0]
    if isinstance(s0, (list, tuple)):
        return type(s0)(map_structure(func, *xs) for xs in zip(*structure))
    if isinstance(s0, dict):
        return {k: map_structure(func, *(s[k] for s in structure)) for k in s0}
    return func(*structure)


def pack_sequence_as(structure, flat_sequence):
    it = iter(flat_sequence)

    def _p(s):
        if isinstance(s, (list, tuple)):
            return type(s)(_p(v) for v in s)
        if isinstance(s, dict):
            return {k: _p(s[k]) for k in sorted(s)}
        return next(it)
    return _p(structure)


def require_version(min_version, max_version=None):
    """Raise if the installed framework version is outside [min_version, max_version]."""
    from .. import __version__ as v

    def key(x):
        return [int(p) if p.isdigit() else 0 for p in str(x).split("+")[0].split(".")][:4]
    if key(v) < key(min_version) or (max_version is not None and key(v) > key(max_version)):
        raise Exception(f"paddlepaddle_amd version {v} does not satisfy [{min_version}, {max_version}]")
