"""MoE expert FFN microbench: grouped HIP GEMM (one launch per projection, device routing) vs the
per-expert loop (host-synced counts + one GEMM per expert). Prints ms and TFLOP/s per config."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from paddlepaddle_amd import ops as O  # noqa: E402
from paddlepaddle_amd.ops import moe as M  # noqa: E402


def loop_ffn(x, eid, w1, w2, K):
    order = torch.argsort(eid, stable=True)
    counts = torch.bincount(eid, minlength=w1.shape[0]).tolist()
    xs = x[order // K]
    outs, off = [], 0
    for e, c in enumerate(counts):
        if c:
            h = O.fused_linear(xs[off:off + c], w1[e], None)
            a, g = h.chunk(2, -1)
            outs.append(O.fused_linear(O.swiglu(a.contiguous(), g.contiguous()), w2[e], None))
        off += c
    return torch.cat(outs)


def grouped_ffn(x, eid, w1, w2, K):
    offs, perm = M.route(eid, w1.shape[0])
    h = M.grouped_linear(x[perm // K], w1, offs)
    a, g = h.chunk(2, -1)
    return M.grouped_linear(O.swiglu(a.contiguous(), g.contiguous()), w2, offs)


def bench(fn, iters=10, bwd=False, params=()):
    for _ in range(2):
        y = fn()
        if bwd:
            y.float().sum().backward()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        y = fn()
        if bwd:
            y.float().sum().backward()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    configs = [("mixtral-like E8 d4096 f14336", 8, 4096, 14336, 8192, 2),
               ("deepseek-like E64 d2048 f1408", 64, 2048, 1408, 8192, 6),
               ("small E64 d1024 f512", 64, 1024, 512, 4096, 2)]
    for name, E, d, f, T, K in configs:
        torch.manual_seed(0)
        x = (torch.randn(T, d, device="cuda") * 0.5).bfloat16()
        w1 = (torch.randn(E, d, 2 * f, device="cuda") * 0.02).bfloat16()
        w2 = (torch.randn(E, f, d, device="cuda") * 0.02).bfloat16()
        logits = torch.randn(T, E, device="cuda")
        eid = logits.topk(K, -1).indices.reshape(-1)
        flops = 2 * T * K * d * (2 * f) + 2 * T * K * f * d
        a = grouped_ffn(x, eid, w1, w2, K)
        b = loop_ffn(x, eid, w1, w2, K)
        err = (a.float() - b.float()).abs().max().item() / (b.float().abs().max().item() + 1e-6)
        tg = bench(lambda: grouped_ffn(x, eid, w1, w2, K))
        tl = bench(lambda: loop_ffn(x, eid, w1, w2, K))
        xg, w1g, w2g = x.clone().requires_grad_(), w1.clone().requires_grad_(), w2.clone().requires_grad_()
        tgb = bench(lambda: grouped_ffn(xg, eid, w1g, w2g, K), bwd=True)
        tlb = bench(lambda: loop_ffn(xg, eid, w1g, w2g, K), bwd=True)
        print(f"{name}: T={T} top{K}  fwd grouped {tg:.2f} ms ({flops / tg / 1e9:.0f} TF)  loop {tl:.2f} ms "
              f"({flops / tl / 1e9:.0f} TF)  speedup {tl / tg:.2f}x | fwd+bwd grouped {tgb:.2f} ms "
              f"({3 * flops / tgb / 1e9:.0f} TF) loop {tlb:.2f} ms ({3 * flops / tlb / 1e9:.0f} TF) "
              f"speedup {tlb / tgb:.2f}x | rel err {err:.3e}", flush=True)


if __name__ == "__main__":
    main()
