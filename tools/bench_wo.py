"""Decode-shape microbench of the weight-only GEMMs (ops/quant.py, csrc/kernels/wo_gemm.hip) against bf16 GEMMs on
the same shapes: hipBLASLt (torch.mm) and this framework's small-M bf16 kernel (ops.gemm.gemm_small_m).
LLaMA-2 7B / GPT-3 13B projection shapes, M = 1 .. 64 rows, median of 3 rounds x 50 launches."""
import sys

import torch

sys.path.insert(0, ".")
import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.nn import quant as Q  # noqa: E402
from paddlepaddle_amd.ops import gemm as G  # noqa: E402
from paddlepaddle_amd.ops import quant as OQ  # noqa: E402


def timeit(fn, iters=50):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def main():
    paddle.set_device("gpu:0")
    shapes = [(4096, 4096), (4096, 11008), (11008, 4096), (5120, 15360), (20480, 5120)]  # (K, N)
    for K, N in shapes:
        w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16) * 0.02
        q8, s8 = [t._t for t in Q.weight_quantize(paddle.Tensor(w.float().cpu()), "weight_only_int8")]
        q4, s4 = [t._t for t in Q.weight_quantize(paddle.Tensor(w.float().cpu()), "weight_only_int4")]
        q8, s8, q4, s4 = q8.cuda(), s8.cuda(), q4.cuda(), s4.cuda()
        for M in (1, 8, 16, 32, 64):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            arms = {"bf16_hipblaslt": lambda: torch.mm(x, w),
                    "int8": lambda: OQ.wo_linear(x, q8, s8, None, 8, -1),
                    "int4": lambda: OQ.wo_linear(x, q4, s4, None, 4, -1)}
            if G.small_m_supported(x, w):
                arms["bf16_ours_small_m"] = lambda: G.gemm_small_m(x, w)
            res = {k: sorted(timeit(f) for _ in range(3))[1] for k, f in arms.items()}
            best_bf16 = min(v for k, v in res.items() if k.startswith("bf16"))
            line = f"K={K:5d} N={N:5d} M={M:2d}: " + "  ".join(f"{k} {v:7.1f}us" for k, v in res.items())
            line += f"  | int8 {best_bf16 / res['int8']:.2f}x  int4 {best_bf16 / res['int4']:.2f}x of best bf16"
            wb = K * N
            line += f"  | int8 weight stream {wb / res['int8'] / 1e6:.2f} TB/s"
            print(line, flush=True)


if __name__ == "__main__":
    main()
