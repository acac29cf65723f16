"""One both-K-major data-gradient shape (LLaMA-2 70B o-projection: M 4096, N 8192, K 8192) on hipBLASLt and on
the hand-written ping-pong (bn 1) and 4-wave (bn 2) kernels, 6 launches each, for rocprofv3 --pmc passes."""
import sys

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import gemm as G  # noqa: E402

M, N, K = 4096, 8192, 8192
dy = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
for _ in range(6):
    torch.mm(dy, w.t())
for _ in range(6):
    G.gemm(dy, w.t(), bn=1)
for _ in range(6):
    G.gemm(dy, w.t(), bn=2)
torch.cuda.synchronize()
