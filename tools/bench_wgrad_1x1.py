"""ResNet-50 1x1-convolution weight gradients (batch 256, NHWC): dW = dY^T . X split-K on the generic kernel
(gemm_splitk) vs the ping-pong 256x256 kernel (gemm_pp_splitk), device time per call."""
import sys

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import conv as C  # noqa: E402
from paddlepaddle_amd.ops import gemm as G  # noqa: E402


def timed(fn, iters=20):
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
    shapes = [(1024, 256, 50176), (256, 1024, 50176), (2048, 512, 12544), (512, 2048, 12544), (1024, 512, 50176),
              (2048, 1024, 12544), (512, 256, 200704), (256, 512, 200704), (512, 1024, 50176)]
    for Cout, Cin, P in shapes:
        dy = torch.randn(P, Cout, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(P, Cin, device="cuda", dtype=torch.bfloat16)
        a = dy.t()
        sp = C._splits(Cout, Cin, P)
        sp2 = G.pp_splits(Cout, Cin, P)
        t1 = timed(lambda: G.gemm_splitk(a, x, sp, out_dtype=torch.bfloat16))
        t2 = timed(lambda: G.gemm_pp_splitk(a, x, sp2, torch.bfloat16)) if G.gemm_pp_splitk_ok(a, x, sp2) else float("nan")
        fl = 2.0 * Cout * Cin * P
        print(f"Cout {Cout:5d} Cin {Cin:5d} P {P:6d}: generic split {sp:3d} {t1:8.1f} us ({fl / t1 / 1e6:5.0f} TF)  "
              f"ping-pong split {sp2:3d} {t2:8.1f} us ({fl / t2 / 1e6:5.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
