"""BN kernels (csrc/kernels/bn.hip) at the ResNet-50 NHWC shapes (batch 256): achieved HBM bandwidth of the
training forward (stats + apply) and backward (reduce + apply), for several reduction grid sizes."""
import sys

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import bn as B  # noqa: E402
from paddlepaddle_amd.ops import _loader as L  # noqa: E402


def timed(fn, it=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1000.0


SHAPES = [(802816, 64), (802816, 256), (200704, 128), (200704, 512), (50176, 256), (50176, 1024), (12544, 512),
          (12544, 2048)]
for wgs in (512, 1024, 2048):
    L.lib().pa_bn_set_target_wgs(wgs)
    tot_f = tot_b = 0.0
    for R, C in SHAPES:
        x = torch.randn(R, C, device="cuda").to(torch.bfloat16).requires_grad_(True)
        res = torch.randn(R, C, device="cuda").to(torch.bfloat16).requires_grad_(True)
        w = torch.ones(C, device="cuda", requires_grad=True)
        b = torch.zeros(C, device="cuda", requires_grad=True)
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        y = B.batch_norm_act_nhwc(x, w, b, rm, rv, True, 0.9, 1e-5, "relu", res)
        g = torch.randn_like(y)
        tf = timed(lambda: B.batch_norm_act_nhwc(x, w, b, rm, rv, True, 0.9, 1e-5, "relu", res))
        tb = timed(lambda: torch.autograd.grad(y, (x, res, w, b), g, retain_graph=True))
        nb = R * C * 2
        tot_f += tf
        tot_b += tb
        print(f"wgs {wgs:5d} R {R:7d} C {C:5d}: fwd {tf:7.1f} us ({3 * nb / tf / 1e3:5.0f} GB/s)  "
              f"bwd {tb:7.1f} us ({7 * nb / tb / 1e3:5.0f} GB/s)", flush=True)
    print(f"wgs {wgs}: total fwd {tot_f:.0f} us, bwd {tot_b:.0f} us", flush=True)
