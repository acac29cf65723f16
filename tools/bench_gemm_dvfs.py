"""GEMM harness reconciliation: the same GPT-3 13B product shapes and layouts as the
training step, hand-written kernel vs hipBLASLt (torch.mm on the same views), timed as sustained loops
(~0.6 s per arm after a 2 s chip warm-up) in interleaved rounds, for several operand distributions:

  uniform  U(-1, 1) bf16 (tools/bench_gemm_abl.py's data)
  train    activations N(0,1), weights N(0, 0.02), output grads N(0, 1e-3)  (what the step multiplies)
  fp8q     N(0,1) rounded to e4m3 and widened to bf16 (tools/bench_fp8.py's bf16 arm: 3-bit mantissas)
  zeros    all-zero operands

MI355X lowers its clock under MFMA load by an amount that depends on the operands' bit activity
(MI355X_MICROARCH.md 'DVFS give-back'), so the same kernel reads different TF/s per distribution."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import gemm as G  # noqa: E402

H, F, Q, T = 5120, 20480, 15360, 4096
# (name, M, N, K, layout) — layout: fwd = x @ W (W [K, N] rows), dgrad = dy @ W^T, wgrad = x^T @ dy
SHAPES = [("qkv", T, Q, H, "fwd"), ("out", T, H, H, "fwd"), ("fc1", T, F, H, "fwd"), ("fc2", T, H, F, "fwd"),
          ("qkv", T, H, Q, "dgrad"), ("out", T, H, H, "dgrad"), ("fc1", T, H, F, "dgrad"), ("fc2", T, F, H, "dgrad"),
          ("qkv", H, Q, T, "wgrad"), ("out", H, H, T, "wgrad"), ("fc1", H, F, T, "wgrad"), ("fc2", F, H, T, "wgrad")]


def fill(shape, mode, role):
    t = torch.empty(shape, device="cuda", dtype=torch.float32)
    if mode == "zeros":
        return t.zero_().bfloat16()
    if mode == "uniform":
        return t.uniform_(-1, 1).bfloat16()
    t.normal_()
    if mode == "fp8q":
        return t.to(torch.float8_e4m3fn).bfloat16()
    scale = {"act": 1.0, "weight": 0.02, "grad": 1e-3}[role]
    return (t * scale).bfloat16()


def operands(M, N, K, layout, mode):
    """(a, b) 2-D views laid out exactly as the step's linear layers hand them to the GEMM."""
    if layout == "fwd":
        return fill((M, K), mode, "act"), fill((K, N), mode, "weight")
    if layout == "dgrad":  # dX[M, K_in=N] = dY[M, N_out=K] @ W^T, W stored [K_in, N_out]
        dy = fill((M, K), mode, "grad")
        w = fill((N, K), mode, "weight")
        return dy, w.t()
    x = fill((K, M), mode, "act")  # wgrad: dW[K_in=M, N_out=N] = X^T @ dY, X [tokens=K, M]
    return x.t(), fill((K, N), mode, "grad")


def sustained(fn, seconds):
    fn()
    torch.cuda.synchronize()
    n, t0 = 0, time.perf_counter()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    while True:
        for _ in range(8):
            fn()
        n += 8
        if n % 32 == 0:
            torch.cuda.synchronize()
            if time.perf_counter() - t0 > seconds:
                break
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=0.6)
    ap.add_argument("--modes", default="uniform,train,fp8q,zeros")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    modes = args.modes.split(",")
    warm = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        torch.mm(warm, warm)
    torch.cuda.synchronize()
    del warm
    tot = {m: {"ours": [0.0, 0.0], "blas": [0.0, 0.0]} for m in modes}  # flops, ms
    for name, M, N, K, layout in SHAPES:
        if args.only and args.only not in f"{layout}:{name}":
            continue
        fl = 2 * M * N * K
        line = f"{layout:5s} {name:3s} M={M:5d} N={N:5d} K={K:5d}"
        for mode in modes:
            a, b = operands(M, N, K, layout, mode)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            arms = {"ours": lambda: G.gemm(a, b, out=out), "blas": lambda: torch.mm(a, b, out=out)}
            best = {k: float("inf") for k in arms}
            for _ in range(args.rounds):
                for k, fn in arms.items():
                    best[k] = min(best[k], sustained(fn, args.seconds))
            for k in arms:
                tot[mode][k][0] += fl
                tot[mode][k][1] += best[k]
            line += f" | {mode}: ours {fl / best['ours'] / 1e9:5.0f} blas {fl / best['blas'] / 1e9:5.0f}"
            del a, b, out
        print(line, flush=True)
    for mode in modes:
        o, b = tot[mode]["ours"], tot[mode]["blas"]
        if o[1]:
            print(f"ALL {mode}: ours {o[0] / o[1] / 1e9:5.0f} TF  blas {b[0] / b[1] / 1e9:5.0f} TF  "
                  f"(sum over shapes)", flush=True)


if __name__ == "__main__":
    main()
