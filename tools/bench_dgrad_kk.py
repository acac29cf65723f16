"""Data-gradient GEMMs dX = dY W^T with paddle's [in, out] weights (both operands K-major) at the GPT-3 13B /
1.3B, LLaMA-2 7B and 70B-layer shapes: hipBLASLt vs the hand-written 256x256 kernels (bn 1 ping-pong, bn 2 4-wave),
operands rotated over 3 buffer sets (> 256 MB MALL) so each call reads cold weights as in a training step.
    PYTHONPATH=. python tools/bench_dgrad_kk.py"""
import torch

from paddlepaddle_amd.ops import gemm as G

SHAPES = {  # name: (M tokens, N = in features, K = out features)
    "13b qkv": (4096, 5120, 15360), "13b o": (4096, 5120, 5120), "13b fc1": (4096, 5120, 20480),
    "13b fc2": (4096, 20480, 5120),
    "1.3b qkv": (8192, 2048, 6144), "1.3b o": (8192, 2048, 2048), "1.3b fc1": (8192, 2048, 8192),
    "1.3b fc2": (8192, 8192, 2048),
    "7b qkv": (8192, 4096, 12288), "7b o": (8192, 4096, 4096), "7b gate_up": (8192, 4096, 22016),
    "7b down": (8192, 11008, 4096),
    "70b qkv": (4096, 8192, 10240), "70b o": (4096, 8192, 8192), "70b gate_up": (4096, 8192, 57344),
    "70b down": (4096, 28672, 8192),
}


def t_us(fn, n=12):
    fn(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n):
        fn(i)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n * 1e3


tot = {"blas": 0.0, "bn1": 0.0, "bn2": 0.0}
for name, (M, N, K) in SHAPES.items():
    dys = [torch.randn(M, K, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(3)]  # W [in, out]
    r = {"blas": t_us(lambda i: torch.mm(dys[i % 3], ws[i % 3].t())),
         "bn1": t_us(lambda i: G.gemm(dys[i % 3], ws[i % 3].t(), bn=1)),
         "bn2": t_us(lambda i: G.gemm(dys[i % 3], ws[i % 3].t(), bn=2))}
    for k in tot:
        tot[k] += r[k]
    fl = 2 * M * N * K
    print(f"{name:12s} M{M} N{N} K{K}: " + "  ".join(f"{k} {v:7.0f}us {fl / v / 1e6:5.0f}TF" for k, v in r.items())
          + f"  hip/blas {min(r['bn1'], r['bn2']) / r['blas']:.3f}", flush=True)
    del dys, ws
print("sum: " + "  ".join(f"{k} {v:.0f}us" for k, v in tot.items()))

# the other two layouts of a training step: forward x @ W (A K-major, B MN-major) and weight gradient x^T dY (both
# MN-major), GPT-3 13B / LLaMA-2 70B shapes
OTHER = {"13b fwd fc1": ("fwd", 4096, 20480, 5120), "13b fwd fc2": ("fwd", 4096, 5120, 20480),
         "70b fwd o": ("fwd", 4096, 8192, 8192), "13b wgrad fc1": ("wgrad", 5120, 20480, 4096),
         "13b wgrad qkv": ("wgrad", 5120, 15360, 4096), "70b wgrad o": ("wgrad", 8192, 8192, 4096)}
for name, (kind, M, N, K) in OTHER.items():
    if kind == "fwd":
        As = [torch.randn(M, K, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
        Bs = [(torch.randn(K, N, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(3)]
    else:  # dW [M = in, N = out] = x^T dY, x [K tokens, in], dY [K, out]
        As = [torch.randn(K, M, device="cuda", dtype=torch.bfloat16).t() for _ in range(3)]
        Bs = [torch.randn(K, N, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    r = {"blas": t_us(lambda i: torch.mm(As[i % 3], Bs[i % 3]))}
    for bn in (1, 2):
        r[f"bn{bn}"] = t_us(lambda i, bn=bn: G.gemm(As[i % 3], Bs[i % 3], bn=bn))
    fl = 2 * M * N * K
    print(f"{name:14s} M{M} N{N} K{K}: " + "  ".join(f"{k} {v:7.0f}us {fl / v / 1e6:5.0f}TF" for k, v in r.items()),
          flush=True)
    del As, Bs
