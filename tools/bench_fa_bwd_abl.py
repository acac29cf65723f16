"""Flash-attention backward ablations (B2 S2048 H40 D128, causal and not): full backward time with
PA_FA_BWD_ABL = 0 (normal), 1 (dQ atomics dropped), 2 (dQ step skipped), 4 (dK/dV GEMMs skipped),
6 (only S / dP / softmax-grad left). Attributes the backward's time to its parts."""
import os
import sys

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import attention as A  # noqa: E402


def main():
    B, S, H, D = 2, 2048, 40, 128
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    for causal in (True, False):
        o = A.flash_attention(q, k, v, causal=causal)
        g = torch.randn_like(o)
        fl = 4 * B * H * S * S * D * (0.5 if causal else 1.0) * 2.5
        for abl in (0, 1, 2, 4, 6):
            os.environ["PA_FA_BWD_ABL"] = str(abl)
            ts = []
            for _ in range(3):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
                torch.cuda.synchronize()
                s.record()
                for _ in range(10):
                    torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) / 10)
            t = min(ts)
            print(f"causal={causal} abl={abl}: {t:.3f} ms  {fl / t / 1e9:.0f} TF (bwd FLOPs = 2.5x fwd)", flush=True)
        os.environ["PA_FA_BWD_ABL"] = "0"


if __name__ == "__main__":
    main()
