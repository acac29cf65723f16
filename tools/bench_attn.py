"""Micro-benchmark: HIP flash attention vs ATen SDPA (aotriton) at GPT shapes. Prints TF/s."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from paddlepaddle_amd.ops.attention import _FlashAttnQKVPackedHIP, _sdpa

def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters

for (B, S, H, D) in [(2, 2048, 40, 128), (8, 2048, 16, 128), (4, 4096, 32, 128), (4, 2048, 32, 64)]:
    qkv = torch.randn(B, S, H, 3, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    flops = 4 * B * H * S * S * D / 2
    o = _FlashAttnQKVPackedHIP.apply(qkv, True, D ** -0.5)
    g = torch.randn_like(o)
    tf = bench(lambda: _FlashAttnQKVPackedHIP.apply(qkv, True, D ** -0.5))
    tb = bench(lambda: torch.autograd.grad(_FlashAttnQKVPackedHIP.apply(qkv, True, D ** -0.5), qkv, g)) - tf
    q, k, v = [qkv[:, :, :, i].detach().contiguous().requires_grad_(True) for i in range(3)]
    rf = bench(lambda: _sdpa(q, k, v, True, D ** -0.5, None, 0.0, False))
    rb = bench(lambda: torch.autograd.grad(_sdpa(q, k, v, True, D ** -0.5, None, 0.0, True), (q, k, v), g)) - rf
    print(f"B{B} S{S} H{H} D{D}: ours fwd {flops/tf/1e12:6.0f} TF bwd {2.5*flops/tb/1e12:6.0f} TF | "
          f"sdpa fwd {flops/rf/1e12:6.0f} TF bwd {2.5*flops/rb/1e12:6.0f} TF", flush=True)
