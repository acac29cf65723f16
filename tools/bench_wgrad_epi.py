"""Weight-gradient GEMMs of the 13B layer: where the time goes. Same product (x^T dy, both operands MN-major)
with the accumulate epilogue (read-modify-write of the bf16 main grad), a plain bf16 store, and the same
product on K-major copies of the operands (layout cost)."""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from paddlepaddle_amd.ops import gemm as G  # noqa: E402
from bench_step_gemms import timed  # noqa: E402


def main():
    dev, bf = "cuda", torch.bfloat16
    w8 = torch.randn(8192, 8192, device=dev, dtype=bf)
    t_end = time.time() + 2.0
    while time.time() < t_end:
        torch.mm(w8, w8)
    T = 4096
    for (I, O) in ((5120, 15360), (5120, 5120), (5120, 20480), (20480, 5120)):
        x = torch.randn(T, I, device=dev, dtype=bf)
        dy = torch.randn(T, O, device=dev, dtype=bf)
        xt, dyt = x.t().contiguous(), dy.t().contiguous()   # [I, T], [O, T]: K-major
        g = torch.zeros(I, O, device=dev, dtype=bf)
        fl = 2 * T * I * O
        r = {
            "MNxMN accum": lambda: G.gemm(x.t(), dy, out=g, accumulate=True),
            "MNxMN store": lambda: G.gemm(x.t(), dy, out=g),
            "KxMN store": lambda: G.gemm(xt, dy, out=g),
            "KxK store": lambda: G.gemm(xt, dyt.t(), out=g),
            "KxK accum": lambda: G.gemm(xt, dyt.t(), out=g, accumulate=True),
        }
        line = []
        for k, f in r.items():
            t = min(timed(f, 20) for _ in range(3))
            line.append(f"{k} {t:7.1f}us {fl / t / 1e6:5.0f}TF")
        print(f"wgrad [{I},{O}] K={T}: " + " | ".join(line), flush=True)


if __name__ == "__main__":
    main()
