"""Flash-attention backward: the 4-wave kernel (fa_bwd_kernel, PA_FA_BWD16=0) vs the 8-wave 16-keys-per-wave
kernel (fa_bwd16_kernel, PA_FA_BWD16=1): time of the whole backward (delta + main kernel + dQ convert) and the max
difference of dQ / dK / dV between the two. TF/s count the backward as 2.5x the forward FLOPs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlepaddle_amd.ops import attention as A  # noqa: E402


def run(B, S, H, Hk, D, causal):
    g0 = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g0).requires_grad_(True)
    k = torch.randn(B, S, Hk, D, device="cuda", dtype=torch.bfloat16, generator=g0).requires_grad_(True)
    v = torch.randn(B, S, Hk, D, device="cuda", dtype=torch.bfloat16, generator=g0).requires_grad_(True)
    o = A.flash_attention(q, k, v, causal=causal)
    g = torch.randn_like(o)
    fl = 4 * B * H * S * S * D * (0.5 if causal else 1.0) * 2.5
    res, grads = {}, {}
    for k16 in ("0", "1"):
        os.environ["PA_FA_BWD16"] = k16
        grads[k16] = torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
        ts = []
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(10):
                torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 10)
        res[k16] = min(ts)
    diff = max((a.float() - b.float()).abs().max().item() for a, b in zip(grads["0"], grads["1"]))
    scale = max(a.float().abs().max().item() for a in grads["0"])
    print(f"B{B} S{S} H{H}/{Hk} D{D} causal={causal}: 4-wave {res['0']:.3f} ms ({fl / res['0'] / 1e9:.0f} TF), "
          f"16-key {res['1']:.3f} ms ({fl / res['1'] / 1e9:.0f} TF), x{res['0'] / res['1']:.2f}, "
          f"max|diff| {diff:.3g} (max |grad| {scale:.3g})", flush=True)


def main():
    for cfg in [(2, 2048, 40, 40, 128, True), (2, 2048, 40, 40, 128, False), (1, 4096, 32, 8, 128, True),
                (4, 1024, 16, 16, 128, True)]:
        run(*cfg)
    os.environ["PA_FA_BWD16"] = "0"


if __name__ == "__main__":
    main()
