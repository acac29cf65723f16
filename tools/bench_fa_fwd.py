"""Flash attention forward: kernel variant 1 (register-staged) vs 2 (glds, 2 LDS stages, deferred
rescale). Checks v2 against v1 and prints TF/s (CUDA events, 20 iterations)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops.attention import _FlashAttnQKVPackedHIP  # noqa: E402

lib = L.lib()
lib.pa_flash_attn_set_fwd_variant.argtypes = [ctypes.c_int]


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it / 1e3


for causal in (True, False):
    for (B, S, H, D) in [(2, 2048, 40, 128), (8, 2048, 16, 128), (4, 4096, 32, 128), (4, 2048, 32, 64),
                         (16, 2048, 64, 128)]:
        qkv = torch.randn(B, S, H, 3, D, device="cuda", dtype=torch.bfloat16)
        flops = 4 * B * H * S * S * D / (2 if causal else 1)
        res = {}
        for v in (1, 2):
            lib.pa_flash_attn_set_fwd_variant(v)
            with torch.no_grad():
                out = _FlashAttnQKVPackedHIP.apply(qkv, causal, D ** -0.5)
                t = timed(lambda: _FlashAttnQKVPackedHIP.apply(qkv, causal, D ** -0.5))
            res[v] = (out.float(), t)
        err = (res[1][0] - res[2][0]).abs().max().item()
        print(f"{'causal' if causal else 'full  '} B{B} S{S} H{H} D{D}: v1 {flops / res[1][1] / 1e12:6.0f} TF  "
              f"v2 {flops / res[2][1] / 1e12:6.0f} TF  max|v1-v2| {err:.2e}", flush=True)
        del qkv, res
lib.pa_flash_attn_set_fwd_variant(2)
for (B, S, H, D) in [(2, 2048, 40, 128), (8, 2048, 16, 128), (4, 4096, 32, 128)]:
    qkv = torch.randn(B, S, H, 3, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    flops = 4 * B * H * S * S * D / 2
    o = _FlashAttnQKVPackedHIP.apply(qkv, True, D ** -0.5)
    g = torch.randn_like(o)
    tf = timed(lambda: _FlashAttnQKVPackedHIP.apply(qkv, True, D ** -0.5))
    tb = timed(lambda: torch.autograd.grad(_FlashAttnQKVPackedHIP.apply(qkv, True, D ** -0.5), qkv, g)) - tf
    print(f"causal B{B} S{S} H{H} D{D}: fwd {flops / tf / 1e12:6.0f} TF  bwd {2.5 * flops / tb / 1e12:6.0f} TF",
          flush=True)
