"""Decode GEMM: hand-written small-M kernel vs hipBLASLt for LLaMA-2 7B projections at batch M."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlepaddle_amd.ops import gemm as G  # noqa: E402


def t(fn, it=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for M in (8, 32, 64):
    for K, N in ((4096, 12288), (4096, 4096), (4096, 22016), (11008, 4096), (4096, 32000)):
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(K, N, device="cuda").bfloat16()
        tb = min(t(lambda: torch.mm(x, w)) for _ in range(3))
        tm = min(t(lambda: G.gemm_small_m(x, w)) for _ in range(3))
        err = ((G.gemm_small_m(x, w).float() - torch.mm(x, w).float()).abs().max() / torch.mm(x, w).float().abs().max()).item()
        gb = K * N * 2 / 1e9
        print(f"M={M} K={K} N={N}: hipBLASLt {tb * 1e3:.1f} us ({gb / tb * 1e3:.0f} GB/s) | small-M {tm * 1e3:.1f} us "
              f"({gb / tm * 1e3:.0f} GB/s) x{tb / tm:.2f} err {err:.0e}", flush=True)
