"""paddle._C_ops: the generated eager op entry points of the reference (paddle/fluid/pybind/eager_op_function.cc).
Code that calls ``paddle._C_ops.<op>(...)`` directly is served by the public API function of the same name
(paddle.*, nn.functional, linalg, incubate functional); ``<op>_`` names map to the in-place variant."""
from __future__ import annotations


def __getattr__(name):
    import paddlepaddle_amd as P
    from .nn import functional as F
    from .incubate.nn import functional as IF
    for ns in (P, F, P.linalg, IF, P.fft):
        fn = getattr(ns, name, None)
        if callable(fn):
            return fn
    if name.endswith("_"):
        base = __getattr__(name[:-1])

        def inplace(x, *a, **k):
            out = base(x, *a, **k)
            x._t.copy_(out._t) if hasattr(out, "_t") else None
            return x
        return inplace
    raise AttributeError(f"paddle._C_ops has no op {name!r}")
