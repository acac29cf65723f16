#!/usr/bin/env python3
"""Build the native parts of paddlepaddle_amd in-tree.

* ``paddlepaddle_amd/_C_hip.so``     — every csrc/kernels/*.hip, hipcc --offload-arch=gfx950, C ABI
                                        (loaded with ctypes by paddlepaddle_amd.ops._loader)
* ``paddlepaddle_amd/_C_runtime*.so`` — csrc/runtime/*.cpp, g++ + pybind11 (CPU runtime)

Incremental: an object is rebuilt only when its source or common.h is newer. Parallel compile.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
BUILD = os.path.join(ROOT, "build", "native")
PKG = os.path.join(ROOT, "paddlepaddle_amd")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-Wno-unused-variable"]


def _newer(src_list, out):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise SystemExit(f"build failed: {cmd[-1] if cmd else ''}")
    return r


def build_hip(verbose=False, jobs=None):
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    hdrs = glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.h"))
    os.makedirs(BUILD, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer([s] + hdrs, o):
            todo.append((s, o))
    jobs = jobs or min(8, max(1, os.cpu_count() or 1))
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_run, [hipcc, *HIP_FLAGS, "-c", s, "-o", o]) for s, o in todo]
        for f in futs:
            f.result()
    out = os.path.join(PKG, "_C_hip.so")
    if todo or _newer(objs, out):
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out, *objs, f"-L{ROCM}/lib", "-lamdhip64"])
    if verbose:
        print(f"built {out} ({len(todo)} objects recompiled)")
    return out


def build_runtime(verbose=False):
    import pybind11
    srcs = sorted(s for s in glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.cpp")) if not s.endswith("_hip.cpp"))
    hdrs = glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.h"))
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    out = os.path.join(PKG, "_C_runtime" + suffix)
    if not _newer(srcs + hdrs, out):
        return out
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", *inc, *srcs, "-o", out, "-ldl"])
    if verbose:
        print(f"built {out}")
    return out


def build_alloc(verbose=False):
    """The HIP device allocator (host code, hipMalloc / events) as a PyTorch pluggable allocator library."""
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "runtime", "*_hip.cpp")))
    hdrs = glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.h"))
    out = os.path.join(PKG, "_C_alloc.so")
    if not _newer(srcs + hdrs, out):
        return out
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    _run([hipcc, "-O3", "-std=c++17", "-fPIC", "-shared", *srcs, "-o", out, f"-L{ROCM}/lib", "-lamdhip64"])
    if verbose:
        print(f"built {out}")
    return out


def main():
    verbose = "-v" in sys.argv or True
    build_hip(verbose)
    build_runtime(verbose)
    build_alloc(verbose)


if __name__ == "__main__":
    main()
