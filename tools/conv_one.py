"""Run one kernel repeatedly for PMC passes: skinny 3x3 conv (C = Cout = 64, 56x56, batch 256) or the 1x1
skinny GEMM. Usage: python tools/conv_one.py conv|gemm [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlepaddle_amd.ops import conv as C  # noqa: E402
from paddlepaddle_amd.ops import gemm as G  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "conv"
it = int(sys.argv[2]) if len(sys.argv) > 2 else 10
if what == "conv":
    x = torch.randn(256, 56, 56, 64, device="cuda").bfloat16()
    wk = (torch.randn(64, 3, 3, 64, device="cuda") * 0.05).bfloat16()
    f = lambda: C._skinny_conv(x, wk, None, 256, 56, 56, 64, 64, 3, 3, 1, 1)  # noqa: E731
else:
    a = torch.randn(256 * 56 * 56, 64, device="cuda").bfloat16()
    b = torch.randn(64, 64, device="cuda").bfloat16().t()
    f = lambda: G.gemm_skinny(a, b)  # noqa: E731
for _ in range(it):
    f()
torch.cuda.synchronize()
print("ok", what)
