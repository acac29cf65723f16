"""fp8 GEMM microbench: hand-written block-scaled-MFMA kernel (ops.fp8.gemm_fp8) vs hipBLASLt fp8
(torch._scaled_mm) vs bf16 hipBLASLt (torch.mm), same shapes, interleaved, best of 3 rounds of 20."""
import sys

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import fp8 as F8  # noqa: E402
from paddlepaddle_amd.ops.fp8 import gemm_fp8  # noqa: E402


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


def main():
    shapes = [(4096, 15360, 5120), (4096, 5120, 5120), (4096, 20480, 5120), (4096, 5120, 20480), (8192, 8192, 8192),
              (16384, 16384, 16384)]
    one = torch.ones((), device="cuda")
    for M, N, K in shapes:
        a = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
        b = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
        a16, b16 = a.to(torch.bfloat16), b.to(torch.bfloat16)
        fl = 2 * M * N * K
        mine = lambda: gemm_fp8(a, b, None, 1.0, "identity", torch.bfloat16)  # noqa: E731
        blas8 = lambda: torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)  # noqa: E731
        bf16 = lambda: torch.mm(a16, b16.t())  # noqa: E731
        ref = (a.float() @ b.float().t())
        err = ((mine().float() - ref).abs().max() / ref.abs().max()).item()
        del ref
        res = {"mine": [], "mine_generic": [], "hipblaslt_fp8": [], "hipblaslt_bf16": []}
        for _ in range(3):
            res["mine"].append(timeit(mine))
            F8.set_kernel("generic")
            res["mine_generic"].append(timeit(mine))
            F8.set_kernel("auto")
            try:
                res["hipblaslt_fp8"].append(timeit(blas8))
            except RuntimeError as ex:
                res["hipblaslt_fp8"].append(float("nan"))
                print("  _scaled_mm failed:", str(ex)[:120])
            res["hipblaslt_bf16"].append(timeit(bf16))
        line = f"M={M} N={N} K={K}:"
        for k, v in res.items():
            t = min(v)
            line += f" {k} {fl / t / 1e9:6.0f} TF ({t:.3f} ms)"
        print(line + f" | err {err:.1e}", flush=True)
        del a, b, a16, b16


if __name__ == "__main__":
    main()
