"""Weight-gradient GEMM layout A/B for the GPT-3 13B linears (mb 2 x seq 2048 = 4096 tokens): dW += X^T dY with
X read in place (A operand MN-major: the both-MN-major kernel) vs X transposed first into a [in, tokens] copy
(A K-major: the forward-layout kernel) + the transpose's own cost. Accumulates into a bf16 gradient buffer the
way the training step does (main-grad fusion).

    python tools/bench_wgrad_layout.py [iters]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import gemm as G  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev, bf = "cuda", torch.bfloat16
    torch.manual_seed(0)
    w8 = torch.randn(8192, 8192, device=dev, dtype=bf)
    t_end = time.time() + 2.0
    while time.time() < t_end:
        torch.mm(w8, w8)
    del w8
    T = 4096
    shapes = [("qkv", 5120, 15360), ("out", 5120, 5120), ("fc1", 5120, 20480), ("fc2", 20480, 5120)]
    tot = {"inplace": 0.0, "transposed": 0.0, "transpose": 0.0}
    for name, K, N in shapes:
        x = torch.randn(T, K, device=dev, dtype=bf)
        dy = torch.randn(T, N, device=dev, dtype=bf) * 1e-3
        acc = torch.zeros(K, N, device=dev, dtype=bf)
        xt_buf = torch.empty(K, T, device=dev, dtype=bf)
        fl = 2.0 * T * K * N
        t_in = timed(lambda: G.gemm(x.t(), dy, out=acc, accumulate=True), iters)
        xt_buf.copy_(x.t())
        t_tg = timed(lambda: G.gemm(xt_buf, dy, out=acc, accumulate=True), iters)
        t_tr = timed(lambda: xt_buf.copy_(x.t()), iters)
        # the transposed-operand product must equal the in-place one
        a1 = torch.zeros_like(acc)
        a2 = torch.zeros_like(acc)
        G.gemm(x.t(), dy, out=a1, accumulate=True)
        G.gemm(xt_buf, dy, out=a2, accumulate=True)
        err = (a1.float() - a2.float()).abs().max().item()
        print(f"{name:4s} [{K}x{N}x{T}] in-place {t_in:7.1f} us ({fl / t_in / 1e6:6.0f} TF)  transposed-A "
              f"{t_tg:7.1f} us ({fl / t_tg / 1e6:6.0f} TF) + transpose {t_tr:6.1f} us  = {t_tg + t_tr:7.1f} us  "
              f"max|diff| {err:.2e}", flush=True)
        tot["inplace"] += t_in
        tot["transposed"] += t_tg
        tot["transpose"] += t_tr
    print(f"layer sum: in-place {tot['inplace']:.0f} us, transposed-A {tot['transposed']:.0f} + transposes "
          f"{tot['transpose']:.0f} = {tot['transposed'] + tot['transpose']:.0f} us", flush=True)


if __name__ == "__main__":
    main()
