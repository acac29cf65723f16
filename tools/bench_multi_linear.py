"""Sibling linears of one input (LLaMA-2 7B q/k/v and gate/up, 8192 tokens): ops.multi_linear (one N-segmented
forward GEMM + one K-segmented data-gradient GEMM) against separate fused_linear calls, forward + backward, and
the two halves split: forward only / data gradient only.

    python tools/bench_multi_linear.py
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import gemm as G  # noqa: E402
from paddlepaddle_amd.ops import linear as LIN  # noqa: E402


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters * 1e3)
    return best


def main():
    dev, bf = "cuda", torch.bfloat16
    torch.manual_seed(0)
    w8 = torch.randn(8192, 8192, device=dev, dtype=bf)
    t_end = time.time() + 2.0
    while time.time() < t_end:
        torch.mm(w8, w8)
    del w8
    T, H = 8192, 4096
    for name, widths in (("qkv", [4096, 4096, 4096]), ("gate_up", [11008, 11008])):
        x = torch.randn(T, H, device=dev, dtype=bf, requires_grad=True)
        ws = [(torch.randn(H, n, device=dev, dtype=bf) * 0.02).requires_grad_(True) for n in widths]
        dys = [torch.randn(T, n, device=dev, dtype=bf) for n in widths]
        fl = 2 * T * H * sum(widths)

        def sep():
            ys = [LIN.fused_linear(x, w) for w in ws]
            torch.autograd.backward(ys, dys)

        def fused():
            ys = LIN.multi_linear(x, ws)
            torch.autograd.backward(ys, dys)

        def fwd_sep():
            with torch.no_grad():
                for w in ws:
                    LIN.fused_linear(x, w)

        def fwd_fused():
            G.gemm_nseg(x.detach(), [w.detach() for w in ws])

        wts = [w.detach().t() for w in ws]

        def dx_sep():
            acc = G.gemm(dys[0], wts[0]) if G.supported(dys[0], wts[0]) else dys[0] @ wts[0]
            for d, wt in zip(dys[1:], wts[1:]):
                acc = acc + (G.gemm(d, wt) if G.supported(d, wt) else d @ wt)

        def dx_blas():
            acc = dys[0] @ wts[0]
            for d, wt in zip(dys[1:], wts[1:]):
                acc.addmm_(d, wt)

        def dx_fused():
            G.gemm_kseg(dys, wts)
        r = {k: timed(f) for k, f in (("fwd+bwd separate", sep), ("fwd+bwd multi_linear", fused),
                                      ("fwd separate", fwd_sep), ("fwd nseg", fwd_fused),
                                      ("dgrad ours separate", dx_sep), ("dgrad hipBLASLt addmm", dx_blas),
                                      ("dgrad kseg", dx_fused))}
        for k, us in r.items():
            tf = (3 if k.startswith("fwd+bwd") else 1) * fl / us / 1e6
            print(f"{name:8s} {k:24s} {us:9.1f} us  {tf:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
