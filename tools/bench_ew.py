"""Elementwise epilogue kernels at the GPT-3 13B MLP shape [4096, 20480] bf16: bias+GELU forward / backward."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from paddlepaddle_amd.ops import activation as A  # noqa: E402
from paddlepaddle_amd.ops import _loader as L  # noqa: E402


def timed(fn, it=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


R, C = 4096, 20480
h = torch.randn(R, C, device="cuda").to(torch.bfloat16)
b = torch.randn(C, device="cuda").to(torch.bfloat16)
dy = torch.randn(R, C, device="cuda").to(torch.bfloat16)
y = torch.empty_like(h)
t = timed(lambda: L.call("pa_bias_gelu_fwd", L.ptr(h), L.ptr(b), L.ptr(y), R, C, L.dcode(h), L.stream_ptr()))
ref = torch.nn.functional.gelu(h.float() + b.float(), approximate="tanh")
print(f"bias_gelu_fwd: {t:6.1f} us ({4 * R * C / t / 1e3:5.0f} GB/s)  max err {(y.float() - ref).abs().max().item():.3e}")
dh = torch.empty_like(h)
db = torch.empty(C, device="cuda", dtype=torch.bfloat16)
ws = torch.empty(256 * C, dtype=torch.float32, device="cuda")
t = timed(lambda: L.call("pa_bias_gelu_bwd", L.ptr(h), L.ptr(b), L.ptr(dy), L.ptr(dh), L.ptr(db), L.ptr(ws), R, C,
                         L.dcode(h), L.stream_ptr()))
print(f"bias_gelu_bwd: {t:6.1f} us ({6 * R * C / t / 1e3:5.0f} GB/s)")

from paddlepaddle_amd.ops import norm as Nm  # noqa: E402
x = torch.randn(4096, 5120, device="cuda").to(torch.bfloat16).requires_grad_(True)
w = torch.rand(5120, device="cuda").to(torch.bfloat16).requires_grad_(True)
bb = torch.randn(5120, device="cuda").to(torch.bfloat16).requires_grad_(True)
yy = Nm._LayerNormHIP.apply(x, w, bb, 1e-5)
g = torch.randn_like(yy)
tf = timed(lambda: Nm._LayerNormHIP.apply(x, w, bb, 1e-5), 20)
tb = timed(lambda: torch.autograd.grad(Nm._LayerNormHIP.apply(x, w, bb, 1e-5), (x, w, bb), g), 20) - tf
print(f"layer_norm [4096, 5120]: fwd {tf:6.1f} us  bwd {tb:6.1f} us")
