"""hipBLASLt vs rocBLAS (torch preferred_blas_library) on the GPT-3 13B GEMM shapes, all three products."""
import torch


def t(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


M = 4096
for K, N in ((5120, 15360), (5120, 5120), (5120, 20480), (20480, 5120)):
    x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    w = torch.empty(K, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    dy = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    acc = torch.zeros(K, N, device="cuda", dtype=torch.bfloat16)
    fl = 2 * M * N * K
    for name, fn in (("fwd", lambda: torch.mm(x, w)), ("dgrad", lambda: torch.mm(dy, w.t())),
                     ("wgrad", lambda: torch.mm(x.t(), dy)), ("wgrad_acc", lambda: acc.addmm_(x.t(), dy))):
        res = {}
        for lib in ("cublaslt", "cublas", "cublaslt", "cublas"):
            torch.backends.cuda.preferred_blas_library(lib)
            res.setdefault(lib, []).append(t(fn))
        torch.backends.cuda.preferred_blas_library("cublaslt")
        a, b = min(res["cublaslt"]), min(res["cublas"])
        print(f"K={K} N={N} {name:9s}: hipBLASLt {fl / a / 1e9:5.0f} TF | rocBLAS {fl / b / 1e9:5.0f} TF  x{a / b:.2f}",
              flush=True)
