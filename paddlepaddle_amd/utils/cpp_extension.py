"""Custom operators. Reference: python/paddle/utils/cpp_extension/ (setup / load / CppExtension /
CUDAExtension building PD_BUILD_OP sources).

MI355X-native form: sources are HIP/C++ compiled by ``hipcc --offload-arch=gfx950`` into a
shared object exporting plain C launchers; ``load`` returns a ctypes handle and
``register_custom_op`` wires a Python forward/backward over them into autograd.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

import torch

from ..framework.tensor import Tensor, _wrap

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def get_build_directory(verbose=False):
    d = os.environ.get("PADDLE_EXTENSION_DIR", os.path.join(os.path.expanduser("~"), ".cache", "paddle_amd_ext"))
    os.makedirs(d, exist_ok=True)
    return d


class CppExtension:
    def __init__(self, sources, *args, **kwargs):
        self.sources = sources
        self.extra_compile_args = kwargs.get("extra_compile_args", {})


CUDAExtension = CppExtension
HIPExtension = CppExtension


def compile_shared(sources, out_path, extra_flags=(), verbose=False):
    hip = any(s.endswith((".hip", ".cu")) for s in sources)
    cc = os.path.join(ROCM, "bin", "hipcc") if hip else "g++"
    cmd = [cc, "-O3", "-fPIC", "-shared", "-std=c++17", "-o", out_path] + list(sources) + list(extra_flags)
    if hip:
        cmd.insert(1, f"--offload-arch={ARCH}")
        cmd += [f"-L{ROCM}/lib", "-lamdhip64"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return out_path


def load(name, sources, extra_cxx_cflags=None, extra_cuda_cflags=None, extra_ldflags=None, extra_include_paths=None,
         build_directory=None, verbose=False):
    build_directory = build_directory or get_build_directory()
    h = hashlib.sha1()
    for s in sources:
        with open(s, "rb") as f:
            h.update(f.read())
    out = os.path.join(build_directory, f"{name}_{h.hexdigest()[:12]}.so")
    if not os.path.exists(out):
        flags = list(extra_cxx_cflags or []) + list(extra_cuda_cflags or []) + list(extra_ldflags or [])
        flags += [f"-I{p}" for p in (extra_include_paths or [])]
        compile_shared(sources, out, flags, verbose)
    import torch  # noqa: F401  (bind to torch's HIP runtime first)
    return ctypes.CDLL(out)


def setup(**attrs):
    exts = attrs.get("ext_modules", [])
    name = attrs.get("name", "custom_op")
    if not isinstance(exts, (list, tuple)):
        exts = [exts]
    outs = []
    for e in exts:
        outs.append(load(name, e.sources))
    return outs


def register_custom_op(name, forward, backward=None):
    """Wrap python callables over raw launchers into a differentiable paddle op."""

    class _Op(torch.autograd.Function):
        @staticmethod
        def forward(ctx, *args):
            ctx.save_for_backward(*[a for a in args if isinstance(a, torch.Tensor)])
            outs = forward(*args)
            return outs

        @staticmethod
        def backward(ctx, *grads):
            if backward is None:
                raise RuntimeError(f"custom op {name} has no backward")
            return backward(ctx.saved_tensors, *grads)

    def op(*args):
        r = _Op.apply(*[a._t if isinstance(a, Tensor) else a for a in args])
        if isinstance(r, tuple):
            return tuple(_wrap(x) for x in r)
        return _wrap(r)
    op.__name__ = name
    return op
