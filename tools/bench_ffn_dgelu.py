"""A/B of the GPT FFN hidden-layer backward: fc2 data-gradient GEMM + GELU backward + fc1 bias gradient, as
(a) hipBLASLt dgrad + pa_bias_gelu_bwd (the split path) and (b) the hand-written GEMM with the GELU backward and
the column sums in its epilogue (pa_gemm_bf16_dgelu, kernels 1 / 2). GPT-3 13B / 1.3B shapes.
Usage: python tools/bench_ffn_dgelu.py"""
import torch

from paddlepaddle_amd.ops import _loader as L
from paddlepaddle_amd.ops import gemm as G
from paddlepaddle_amd.ops import linear as LIN


def t_ms(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


for M, H, F in ((4096, 5120, 20480), (8192, 2048, 8192), (4096, 4096, 16384)):
    dy = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
    w2 = (torch.randn(F, H, device="cuda") * 0.02).to(torch.bfloat16)
    pre = torch.randn(M, F, device="cuda", dtype=torch.bfloat16)
    zb = torch.zeros(F, device="cuda", dtype=torch.bfloat16)
    w2t = w2.t()
    res = {}
    res["blas_mm"] = t_ms(lambda: torch.mm(dy, w2t))
    res["split(blas+bias_gelu_bwd)"] = t_ms(lambda: LIN._bias_gelu_bwd(pre, zb, torch.mm(dy, w2t)))
    res["hip_mm_pp"] = t_ms(lambda: G.gemm(dy, w2t, bn=1))
    for k in (1, 2):
        res[f"fused_k{k}"] = t_ms(lambda k=k: G.gemm_dgelu(dy, w2t, pre, k))
    fl = 2 * M * H * F
    print(f"M{M} H{H} F{F}: " + "  ".join(f"{n} {v * 1e3:.0f}us ({fl / v / 1e9:.0f} TF)" for n, v in res.items()),
          flush=True)

# weight gradients accumulated into an fp32 / bf16 main-grad buffer (the accumulate epilogue's read-ahead)
for K, Mw, Nw in ((4096, 5120, 20480), (4096, 20480, 5120), (4096, 5120, 15360)):
    x = torch.randn(K, Mw, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(K, Nw, device="cuda", dtype=torch.bfloat16)
    for dt in (torch.float32, torch.bfloat16):
        acc = torch.zeros(Mw, Nw, device="cuda", dtype=dt)
        res = {"hip_acc": t_ms(lambda: G.gemm(x.t(), dy, out=acc, accumulate=True, bn=1)),
               "blas_addmm": t_ms(lambda: acc.addmm_(x.t(), dy)) if dt == torch.bfloat16 else float("nan"),
               "hip_noacc": t_ms(lambda: G.gemm(x.t(), dy, bn=1))}
        fl = 2 * K * Mw * Nw
        print(f"wgrad {Mw}x{Nw}x{K} acc {dt}: " + "  ".join(f"{n} {v * 1e3:.0f}us ({fl / v / 1e9:.0f} TF)"
                                                           for n, v in res.items()), flush=True)
