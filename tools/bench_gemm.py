"""GEMM layout microbenchmark: y = x @ W with W stored [in, out] (NN) vs [out, in] (TN), for the
GPT-3 13B linear shapes. Prints TFLOP/s per variant."""
import torch


def bench(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dt = torch.bfloat16
    for M in (4096, 8192):
        for K, N in ((5120, 15360), (5120, 5120), (5120, 20480), (20480, 5120)):
            x = torch.randn(M, K, device="cuda", dtype=dt)
            w = torch.randn(K, N, device="cuda", dtype=dt)
            wt = w.t().contiguous()
            dy = torch.randn(M, N, device="cuda", dtype=dt)
            fl = 2 * M * N * K
            r = {}
            r["fwd_NN"] = bench(lambda: torch.matmul(x, w))
            r["fwd_TN"] = bench(lambda: torch.matmul(x, wt.t()))
            r["dgrad_w[in,out]"] = bench(lambda: torch.matmul(dy, w.t()))
            r["dgrad_w[out,in]"] = bench(lambda: torch.matmul(dy, wt))
            r["wgrad x^T dy"] = bench(lambda: torch.matmul(x.t(), dy))
            r["wgrad dy^T x"] = bench(lambda: torch.matmul(dy.t(), x))
            print(f"M={M} K={K} N={N}: " + "  ".join(f"{k}={fl / v / 1e9:.0f}TF({v:.3f}ms)" for k, v in r.items()),
                  flush=True)


if __name__ == "__main__":
    main()
