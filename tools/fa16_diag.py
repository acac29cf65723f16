"""Diagnostics of the 16-keys-per-wave flash-attention backward (PA_FA_BWD16 levels): 1 normal (vs the 4-wave
kernel), 2 no dQ step, 3 P := 1 (dV = column sums of dO), 4 P := S' (raw QK^T - lse/scale accumulator)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlepaddle_amd.ops import attention as A  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 32
torch.manual_seed(0)
q, k, v = (torch.randn(1, S, 1, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
o, lse = A.flash_attention(q, k, v, causal=False), None
g = torch.randn_like(o)
os.environ["PA_FA_BWD16"] = "0"
ref = torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
for lvl in ("1", "2", "3", "4"):
    os.environ["PA_FA_BWD16"] = lvl
    got = torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
    torch.cuda.synchronize()
    dv = got[2][0, :, 0].float()
    line = f"level {lvl}: nan dq/dk/dv {[bool(t.isnan().any()) for t in got]}"
    if lvl in ("1", "2"):
        line += f" dv err {(dv - ref[2][0, :, 0].float()).abs().max().item():.3g}"
    if lvl == "3":
        exp = g[0, :, 0].float().sum(0, keepdim=True).expand(S, 128)
        line += f" dv vs colsum(dO) err {(dv - exp).abs().max().item():.3g} (max {exp.abs().max().item():.3g})"
        line += f" dv[0,:4] {dv[0, :4].tolist()} exp {exp[0, :4].tolist()}"
    if lvl == "4":
        scale = 128 ** -0.5
        sp = q[0, :, 0].float() @ k[0, :, 0].float().T  # S' without the lse term: compare shapes only
        line += f" dv[0,:4] {dv[0, :4].tolist()}"
    print(line, flush=True)
os.environ["PA_FA_BWD16"] = "0"
