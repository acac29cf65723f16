"""ResNet-50 3x3 conv weight gradient: split-K implicit GEMM (ours) vs MIOpen (aten convolution_backward)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from paddlepaddle_amd.ops import conv as Cv  # noqa: E402


def timed(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


B = 256
for (H, C, stride) in [(56, 64, 1), (56, 128, 2), (28, 128, 1), (28, 256, 2), (14, 256, 1), (14, 512, 2), (7, 512, 1)]:
    Ho = H // stride
    x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
    dy = torch.randn(B, Ho, Ho, C, device="cuda").to(torch.bfloat16)
    w = torch.randn(C, C, 3, 3, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    fl = 2 * B * Ho * Ho * 9 * C * C

    def ours():
        return Cv._implicit_wgrad(x, dy, w, B, H, H, C, C, 3, 3, stride, 1, 1, Ho, Ho)

    def miopen():
        return torch.ops.aten.convolution_backward(dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w, None,
                                                   [stride] * 2, [1, 1], [1, 1], False, [0, 0], 1,
                                                   [False, True, False])[1]
    a, b = ours(), miopen()
    err = ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
    to, tm = timed(ours), timed(miopen)
    print(f"H{H} C{C} s{stride}: ours {to * 1e3:7.1f} us ({fl / to / 1e9:5.0f} TF) | MIOpen {tm * 1e3:7.1f} us "
          f"({fl / tm / 1e9:5.0f} TF) x{tm / to:.2f} relerr {err:.1e} splits {Cv._wgrad_splits(B * Ho * Ho, 9 * C, C, 256 if C % 256 == 0 else (64 if C <= 64 else 128))}",
          flush=True)
