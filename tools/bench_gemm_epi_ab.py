"""Staged-epilogue GEMMs (accumulate into an fp32 / bf16 main-grad buffer, plain bf16) at the GPT-3 13B
weight-gradient shapes, cold operands (each rep reads new buffers: no MALL reuse of the accumulator).
Run once per build to A/B an epilogue change: PYTHONPATH=<tree> python tools/bench_gemm_epi_ab.py"""
import torch

from paddlepaddle_amd.ops import gemm as G


def t_ms(fn, n=12):
    fn(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n):
        fn(i)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


for K, Mw, Nw in ((4096, 5120, 20480), (4096, 20480, 5120), (4096, 5120, 15360), (4096, 5120, 5120)):
    x = torch.randn(K, Mw, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(K, Nw, device="cuda", dtype=torch.bfloat16)
    out = []
    for dt in (torch.float32, torch.bfloat16):
        accs = [torch.zeros(Mw, Nw, device="cuda", dtype=dt) for _ in range(3)]  # rotate: 3 x 400 MB > MALL
        out.append(f"acc_{str(dt)[6:]} {t_ms(lambda i: G.gemm(x.t(), dy, out=accs[i % 3], accumulate=True, bn=1)) * 1e3:.0f}us")
        del accs
    out.append(f"plain {t_ms(lambda i: G.gemm(x.t(), dy, bn=1)) * 1e3:.0f}us")
    print(f"wgrad {Mw}x{Nw}x{K}: " + "  ".join(out), flush=True)
