"""The GEMMs of one GPT-3 13B decoder layer x micro-batch (mb 2 x seq 2048 = 4096 tokens), each with the epilogue
the training step uses, timed back to back on training-like operands: hand-written kernel vs hipBLASLt (+ the
separate pass that the vendor path needs for the same epilogue). Prints per-shape device time and the layer sum.

    python tools/bench_step_gemms.py [iters]
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
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev, bf = "cuda", torch.bfloat16
    torch.manual_seed(0)
    w8 = torch.randn(8192, 8192, device=dev, dtype=bf)
    t_end = time.time() + 2.0
    while time.time() < t_end:  # settle the clock under sustained load
        torch.mm(w8, w8)
    del w8
    T, H, F, Q = 4096, 5120, 20480, 15360
    x = torch.randn(T, H, device=dev, dtype=bf)
    xf = torch.randn(T, F, device=dev, dtype=bf)
    w_qkv = torch.randn(H, Q, device=dev, dtype=bf) * 0.02
    w_o = torch.randn(H, H, device=dev, dtype=bf) * 0.02
    w_1 = torch.randn(H, F, device=dev, dtype=bf) * 0.02
    w_2 = torch.randn(F, H, device=dev, dtype=bf) * 0.02
    b_q, b_h, b_f = (torch.randn(n, device=dev, dtype=bf) * 0.02 for n in (Q, H, F))
    dy_q, dy_h, dy_f = (torch.randn(T, n, device=dev, dtype=bf) for n in (Q, H, F))
    pre = torch.empty(T, F, device=dev, dtype=bf)
    g_qkv, g_o, g_1, g_2 = (torch.zeros_like(w) for w in (w_qkv, w_o, w_1, w_2))

    def gelu_pass(h):
        return torch.nn.functional.gelu(h + b_f, approximate="tanh")
    cases = [
        ("fwd qkv", 2 * T * Q * H, lambda: G.gemm(x, w_qkv, bias=b_q), lambda: torch.addmm(b_q, x, w_qkv)),
        ("fwd out", 2 * T * H * H, lambda: G.gemm(x, w_o, bias=b_h), lambda: torch.addmm(b_h, x, w_o)),
        ("fwd fc1+gelu", 2 * T * F * H, lambda: G.gemm(x, w_1, bias=b_f, gelu=True, aux=pre),
         lambda: gelu_pass(torch.mm(x, w_1))),
        ("fwd fc2", 2 * T * H * F, lambda: G.gemm(xf, w_2, bias=b_h), lambda: torch.addmm(b_h, xf, w_2)),
        ("dgrad fc2", 2 * T * F * H, lambda: G.gemm(dy_h, w_2.t()), lambda: torch.mm(dy_h, w_2.t())),
        ("dgrad fc1", 2 * T * H * F, lambda: G.gemm(dy_f, w_1.t()), lambda: torch.mm(dy_f, w_1.t())),
        ("dgrad out", 2 * T * H * H, lambda: G.gemm(dy_h, w_o.t()), lambda: torch.mm(dy_h, w_o.t())),
        ("dgrad qkv", 2 * T * H * Q, lambda: G.gemm(dy_q, w_qkv.t()), lambda: torch.mm(dy_q, w_qkv.t())),
        ("wgrad qkv", 2 * T * H * Q, lambda: G.gemm(x.t(), dy_q, out=g_qkv, accumulate=True),
         lambda: g_qkv.addmm_(x.t(), dy_q)),
        ("wgrad out", 2 * T * H * H, lambda: G.gemm(x.t(), dy_h, out=g_o, accumulate=True),
         lambda: g_o.addmm_(x.t(), dy_h)),
        ("wgrad fc1", 2 * T * H * F, lambda: G.gemm(x.t(), dy_f, out=g_1, accumulate=True),
         lambda: g_1.addmm_(x.t(), dy_f)),
        ("wgrad fc2", 2 * T * F * H, lambda: G.gemm(xf.t(), dy_h, out=g_2, accumulate=True),
         lambda: g_2.addmm_(xf.t(), dy_h)),
    ]
    only = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else None
    tot_h = tot_b = tot_best = 0.0
    for name, fl, f_h, f_b in cases:
        if only and name.split()[0] not in only:
            continue
        th = min(timed(f_h, iters) for _ in range(3))
        tb = min(timed(f_b, iters) for _ in range(3))
        tot_h += th
        tot_b += tb
        tot_best += min(th, tb)
        print(f"{name:14s} ours {th:8.1f} us {fl / th / 1e6:6.0f} TF | blas {tb:8.1f} us {fl / tb / 1e6:6.0f} TF | "
              f"ours/blas x{tb / th:.3f}", flush=True)
    print(f"layer total: ours {tot_h:.0f} us, blas {tot_b:.0f} us, best-of {tot_best:.0f} us", flush=True)


if __name__ == "__main__":
    main()
