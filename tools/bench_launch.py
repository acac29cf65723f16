"""Host-side cost of one eager HIP-kernel launch through the op layer: the native METH_FASTCALL path
(csrc/dispatch) vs the ctypes path (PADDLE_AMD_CTYPES_LAUNCH=1). Tiny shapes, so the loop is launch-bound.
Usage: python tools/bench_launch.py            (runs both paths in child processes and prints a table)"""
import os
import subprocess
import sys
import time


def _child():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import paddlepaddle_amd  # noqa: F401
    from paddlepaddle_amd.ops import _loader as L
    from paddlepaddle_amd.ops import norm as N
    from paddlepaddle_amd.ops import activation as A
    x = torch.randn(8, 1024, device="cuda", dtype=torch.bfloat16)
    w = torch.ones(1024, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(8, 2048, device="cuda", dtype=torch.bfloat16)
    y = torch.empty_like(x)
    r = torch.empty(8, device="cuda", dtype=torch.float32)
    cases = {
        "rms_norm fwd (9 args)": lambda: N.rms_norm(x, w, 1e-6),
        "swiglu fwd (8 args)": lambda: A.swiglu(g[:, :1024], g[:, 1024:]),
        "raw launcher call (9 args)": lambda: L.call("pa_rms_norm_fwd", L.ptr(x), L.ptr(w), L.ptr(y), L.ptr(r),
                                                     8, 1024, 1e-6, L.dcode(x), L.stream_ptr()),
    }
    mode = "native" if L.native_launch() else "ctypes"
    with torch.no_grad():
        for name, fn in cases.items():
            for _ in range(200):
                fn()
            torch.cuda.synchronize()
            n = 5000
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            print(f"{mode:7s} {name:28s} {(t1 - t0) / n * 1e6:7.2f} us/op (host)", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        _child()
        return
    for env in ({}, {"PADDLE_AMD_CTYPES_LAUNCH": "1"}):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env={**os.environ, **env})
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
