"""The 13B step's flash-attention backward (B4 S2048 H40 D128 causal, dS route) a few times, for rocprofv3 --pmc
passes over fa_bwd16_kernel / fa_bwd_dq_kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from paddlepaddle_amd.ops import attention as A  # noqa: E402

B, S, H, D = 4, 2048, 40, 128
qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
for _ in range(5):
    o = A.flash_attention_qkvpacked(qkv.permute(0, 1, 3, 2, 4), causal=True)
    o.backward(torch.ones_like(o))
torch.cuda.synchronize()
print("ok")
