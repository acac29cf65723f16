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


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def pair_main():
    """Weight-gradient pairing: two K = 4096 accumulating products vs one two-segment K = 8192 product."""
    from paddlepaddle_amd.ops import gemm as G2
    dev, bf = "cuda", torch.bfloat16
    T = 4096
    for (I, O) in ((5120, 15360), (5120, 5120), (5120, 20480), (20480, 5120)):
        xa, xb = (torch.randn(T, I, device=dev, dtype=bf) for _ in range(2))
        da, db = (torch.randn(T, O, device=dev, dtype=bf) for _ in range(2))
        g = torch.zeros(I, O, device=dev, dtype=bf)
        fl = 4 * T * I * O
        t2 = min(timed(lambda: (G2.gemm(xa.t(), da, out=g, accumulate=True),
                                G2.gemm(xb.t(), db, out=g, accumulate=True)), 10) for _ in range(3))
        t1 = min(timed(lambda: G2.gemm_seg(xa.t(), xb.t(), da, db, out=g, accumulate=True), 10) for _ in range(3))
        print(f"wgrad pair [{I},{O}]: 2 x K=4096 {t2:7.1f}us {fl / t2 / 1e6:5.0f}TF | one K=4096+4096 "
              f"{t1:7.1f}us {fl / t1 / 1e6:5.0f}TF | x{t2 / t1:.3f}", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pair":
    pair_main()
