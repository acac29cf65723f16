"""Run one GEMM variant on one shape repeatedly (for rocprofv3 --pmc passes).
Usage: python tools/gemm_one.py <bn> <layout fwd|dgrad|wgrad> [M K N iters]"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from paddlepaddle_amd.ops import gemm as G  # noqa: E402

bn = int(sys.argv[1])
lay = sys.argv[2]
M, K, N, it = (int(v) for v in (sys.argv[3:7] if len(sys.argv) > 6 else (4096, 5120, 20480, 10)))
x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
w = torch.empty(K, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
dy = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
for _ in range(it):
    if bn == 0:
        torch.mm(x, w) if lay == "fwd" else (torch.mm(dy, w.t()) if lay == "dgrad" else torch.mm(x.t(), dy))
    elif lay == "fwd":
        G.gemm(x, w, bn=bn)
    elif lay == "dgrad":
        G.gemm(dy, w.t(), bn=bn)
    else:
        G.gemm(x.t(), dy, bn=bn)
torch.cuda.synchronize()
print("ok")
