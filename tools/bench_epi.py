"""Cost of the fused GEMM epilogues on the ping-pong kernel (fc1 of GPT-3 13B: 4096 x 20480 x 5120)."""
import sys

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import gemm as G  # noqa: E402
from paddlepaddle_amd.ops import _loader as L  # noqa: E402


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


M, K, N = 4096, 5120, 20480
x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
w = torch.empty(K, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
b = torch.empty(N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
acc32 = torch.zeros(M, N, device="cuda", dtype=torch.float32)
cases = {
    "hipBLASLt mm": lambda: torch.mm(x, w),
    "hipBLASLt addmm(bias)": lambda: torch.addmm(b, x, w),
    "pp plain": lambda: G.gemm(x, w, out=out, bn=1),
    "pp bias": lambda: G.gemm(x, w, bias=b, out=out, bn=1),
    "pp bias+gelu": lambda: G.gemm(x, w, bias=b, gelu=True, out=out, bn=1),
    "pp bias+gelu+aux": lambda: G.gemm(x, w, bias=b, gelu=True, aux=aux, out=out, bn=1),
    "pp accum fp32": lambda: G.gemm(x, w, out=acc32, accumulate=True, bn=1),
}
res = {k: [] for k in cases}
for _ in range(3):
    for k, fn in cases.items():
        res[k].append(timeit(fn))
fl = 2 * M * N * K
for k, v in res.items():
    t = min(v)
    print(f"{k:24s} {t:.3f} ms  {fl / t / 1e9:6.0f} TF", flush=True)
