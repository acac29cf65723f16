"""Decode-attention microbenchmark: HBM bandwidth of ops.paged_decode_attention (HIP flash-decoding)
vs the torch gather reference, on LLaMA-style GQA shapes. Usage: python tools/bench_decode.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlepaddle_amd import ops  # noqa: E402
from paddlepaddle_amd.ops.attention import paged_decode_reference  # noqa: E402


def run(N, H, Hkv, ctx, bs=64, iters=50):
    D = 128
    nbps = (ctx + bs - 1) // bs
    kc = torch.randn(N * nbps, Hkv, bs, D, device="cuda").bfloat16()
    vc = torch.randn_like(kc)
    tab = torch.randperm(N * nbps, device="cuda").int().view(N, nbps)
    lens = torch.full((N,), ctx, dtype=torch.int32, device="cuda")
    q = torch.randn(N, H, D, device="cuda").bfloat16()
    f = lambda: ops.paged_decode_attention(q, kc, vc, tab, lens, max_len=ctx)  # noqa: E731
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    gb = 2 * N * ctx * Hkv * D * 2 / 1e9
    line = f"N={N:4d} H={H:3d} Hkv={Hkv:2d} ctx={ctx:6d}: {ms * 1e3:8.1f} us  {gb / ms:7.0f} GB/s (K+V bytes)"
    if N * ctx <= 32 * 4096:
        r = lambda: paged_decode_reference(q, kc, vc, tab, lens)  # noqa: E731
        r()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(5):
            r()
        e1.record()
        torch.cuda.synchronize()
        line += f"   torch-gather {e0.elapsed_time(e1) / 5 * 1e3:9.1f} us"
    print(line, flush=True)


if __name__ == "__main__":
    for N, H, Hkv, ctx in [(1, 32, 8, 4096), (1, 64, 8, 32768), (8, 32, 8, 4096), (32, 32, 8, 2048),
                           (64, 40, 40, 2048), (128, 32, 8, 4096), (256, 64, 8, 1024), (16, 32, 32, 8192)]:
        run(N, H, Hkv, ctx)
