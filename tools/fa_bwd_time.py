"""Time the flash-attention backward at the 13B micro-batch shape (B4 S2048 H40 D128 causal) with hip events;
run once per PA_FA_* setting (the switches are read once per process)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from paddlepaddle_amd.ops import attention as A  # noqa: E402

B, S, H, D = 4, 2048, 40, 128
qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
ts = []
for i in range(25):
    o = A.flash_attention_qkvpacked(qkv.permute(0, 1, 3, 2, 4), causal=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    o.backward(g)
    e1.record()
    torch.cuda.synchronize()
    if i >= 5:
        ts.append(e0.elapsed_time(e1))
ts.sort()
print(f"PA_FA_DQ_SLOTS={os.environ.get('PA_FA_DQ_SLOTS', '4')} bwd median {ts[len(ts) // 2] * 1000:.1f} us "
      f"min {ts[0] * 1000:.1f} us  dq norm {qkv.grad.float().norm().item():.4f}")
