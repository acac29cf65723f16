"""Depthwise NHWC convolution: hand-written HIP kernels (ops/dwconv.py) vs MIOpen (torch conv2d, channels_last),
forward + backward, bf16, MobileNetV2 shapes at batch 128."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from paddlepaddle_amd.ops import dwconv  # noqa: E402

SHAPES = [(128, 112, 112, 32, 1), (128, 112, 112, 96, 2), (128, 56, 56, 144, 1), (128, 56, 56, 144, 2),
          (128, 28, 28, 192, 1), (128, 14, 14, 384, 1), (128, 14, 14, 576, 1), (128, 7, 7, 960, 1)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    for N, H, W, C, s in SHAPES:
        x = torch.randn(N, H, W, C, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        w = (torch.randn(C, 1, 3, 3, device="cuda") * 0.3).to(torch.bfloat16).requires_grad_(True)
        gy = None

        def ours():
            y = dwconv._DWConv.apply(x, w, None, (s, s), (1, 1), (1, 1))
            y.backward(torch.ones_like(y))

        def miopen():
            y = F.conv2d(x.permute(0, 3, 1, 2), w.contiguous(memory_format=torch.channels_last), None, s, 1, 1, C)
            y.backward(torch.ones_like(y))
        a, b = timeit(ours), timeit(miopen)
        Ho = (H - 1) // s + 1
        mb = (N * H * W * C * 2 * 3 + N * Ho * Ho * C * 2 * 3) / 1e6  # x, dx, x again; y, dy twice
        print(f"N{N} {H}x{W} C{C} s{s}: hip {a:.3f} ms ({mb / a:.0f} GB/s eff), MIOpen {b:.3f} ms, x{b / a:.2f}",
              flush=True)


if __name__ == "__main__":
    main()
