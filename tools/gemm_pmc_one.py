"""One GEMM shape on each backend, a few launches each, for rocprofv3 --pmc passes (tools/gpu_r5d.sh)."""
import sys

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import gemm as G  # noqa: E402

T, H, F = 4096, 5120, 20480
dy = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
w2 = torch.randn(F, H, device="cuda", dtype=torch.bfloat16) * 0.02
for _ in range(3):
    G.gemm(dy, w2.t(), bn=1)
    G.gemm(dy, w2.t(), bn=2)
    torch.mm(dy, w2.t())
torch.cuda.synchronize()
