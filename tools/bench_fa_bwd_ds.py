"""Flash-attention backward, D = 128: the atomics kernel (fa_bwd16_kernel + fp32 dQ atomics + convert,
PA_FA_BWD_DS=0) vs the dS route (fa_bwd16_kernel<.., true> writing dS^T tiles + fa_bwd_dq_kernel, PA_FA_BWD_DS=1).
Whole backward (delta + kernels), best of 3 x 10; TF/s count the backward as 2.5x the forward FLOPs. Also prints
the max difference of dQ / dK / dV between the two routes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlepaddle_amd.ops import attention as A  # noqa: E402


def run(B, S, H, Hk, D, causal, reps=10):
    g0 = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g0).requires_grad_(True)
    k = torch.randn(B, S, Hk, D, device="cuda", dtype=torch.bfloat16, generator=g0).requires_grad_(True)
    v = torch.randn(B, S, Hk, D, device="cuda", dtype=torch.bfloat16, generator=g0).requires_grad_(True)
    o = A.flash_attention(q, k, v, causal=causal)
    g = torch.randn_like(o)
    fl = 4 * B * H * S * S * D * (0.5 if causal else 1.0) * 2.5
    res, grads = {}, {}
    for ds in ("0", "1"):
        os.environ["PA_FA_BWD_DS"] = ds
        grads[ds] = torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
        ts = []
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(reps):
                torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / reps)
        res[ds] = min(ts)
    diff = [(a.float() - b.float()).abs().max().item() for a, b in zip(grads["0"], grads["1"])]
    scale = [a.float().abs().max().item() for a in grads["0"]]
    print(f"B{B} S{S} H{H}/{Hk} D{D} causal={causal}: atomics {res['0']:.3f} ms ({fl / res['0'] / 1e9:.0f} TF), "
          f"dS route {res['1']:.3f} ms ({fl / res['1'] / 1e9:.0f} TF), x{res['0'] / res['1']:.2f}; "
          f"max|diff| dq/dk/dv {diff[0]:.3g}/{diff[1]:.3g}/{diff[2]:.3g} (max|grad| {scale[0]:.3g}/{scale[1]:.3g}/"
          f"{scale[2]:.3g})", flush=True)


def main():
    cfgs = [(2, 2048, 40, 40, 128, True), (2, 2048, 40, 40, 128, False), (2, 4096, 32, 32, 128, True),
            (1, 4096, 64, 8, 128, True), (4, 1024, 16, 16, 128, True)]
    if len(sys.argv) > 1 and sys.argv[1] == "headline":
        cfgs = cfgs[:1]
    for cfg in cfgs:
        run(*cfg)
    os.environ.pop("PA_FA_BWD_DS", None)


if __name__ == "__main__":
    main()
