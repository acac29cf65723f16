"""paddle.sysconfig (reference python/paddle/sysconfig.py): where the C/C++ headers and the native
libraries of the framework live, for building custom operators against it."""
import os

_ROOT = os.path.dirname(os.path.abspath(__file__))


def get_include():
    """Directory of the kernel headers (csrc/kernels/common.h) used by custom HIP ops."""
    src = os.path.join(os.path.dirname(_ROOT), "csrc", "kernels")
    return src if os.path.isdir(src) else os.path.join(_ROOT, "include")


def get_lib():
    """Directory holding _C_hip.so / _C_runtime*.so."""
    return _ROOT
