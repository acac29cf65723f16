"""The 13B layer's GEMMs (tools/bench_step_gemms.py shapes and epilogues) on each hand-written 256x256 variant:
bn=1 8-wave ping-pong, bn=2 4-wave K32 ring, plus hipBLASLt; checks each variant against the ping-pong output
first (same operands), then times them back to back.

    python tools/bench_gemm_variants.py [iters] [variants, e.g. 1,2]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from paddlepaddle_amd.ops import gemm as G  # noqa: E402
from bench_step_gemms import timed  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    variants = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2]
    dev, bf = "cuda", torch.bfloat16
    torch.manual_seed(0)
    w8 = torch.randn(8192, 8192, device=dev, dtype=bf)
    t_end = time.time() + 2.0
    while time.time() < t_end:
        torch.mm(w8, w8)
    del w8
    T, H, F, Q = 4096, 5120, 20480, 15360
    x = torch.randn(T, H, device=dev, dtype=bf)
    xf = torch.randn(T, F, device=dev, dtype=bf)
    w_qkv = torch.randn(H, Q, device=dev, dtype=bf) * 0.02
    w_o = torch.randn(H, H, device=dev, dtype=bf) * 0.02
    w_1 = torch.randn(H, F, device=dev, dtype=bf) * 0.02
    w_2 = torch.randn(F, H, device=dev, dtype=bf) * 0.02
    b_q, b_h, b_f = (torch.randn(n, device=dev, dtype=bf) * 0.02 for n in (Q, H, F))
    dy_q, dy_h, dy_f = (torch.randn(T, n, device=dev, dtype=bf) for n in (Q, H, F))
    pre = torch.empty(T, F, device=dev, dtype=bf)
    g_qkv, g_o, g_1, g_2 = (torch.zeros_like(w) for w in (w_qkv, w_o, w_1, w_2))
    def gelu_pass(h):
        return torch.nn.functional.gelu(h + b_f, approximate="tanh")
    blas = {
        "fwd qkv": lambda: torch.addmm(b_q, x, w_qkv), "fwd out": lambda: torch.addmm(b_h, x, w_o),
        "fwd fc1+gelu": lambda: gelu_pass(torch.mm(x, w_1)), "fwd fc2": lambda: torch.addmm(b_h, xf, w_2),
        "dgrad fc2": lambda: torch.mm(dy_h, w_2.t()), "dgrad fc1": lambda: torch.mm(dy_f, w_1.t()),
        "dgrad out": lambda: torch.mm(dy_h, w_o.t()), "dgrad qkv": lambda: torch.mm(dy_q, w_qkv.t()),
        "wgrad qkv": lambda: g_qkv.addmm_(x.t(), dy_q), "wgrad out": lambda: g_o.addmm_(x.t(), dy_h),
        "wgrad fc1": lambda: g_1.addmm_(x.t(), dy_f), "wgrad fc2": lambda: g_2.addmm_(xf.t(), dy_h),
    }
    cases = [
        ("fwd qkv", 2 * T * Q * H, lambda bn, o=None: G.gemm(x, w_qkv, bias=b_q, bn=bn, out=o)),
        ("fwd out", 2 * T * H * H, lambda bn, o=None: G.gemm(x, w_o, bias=b_h, bn=bn, out=o)),
        ("fwd fc1+gelu", 2 * T * F * H, lambda bn, o=None: G.gemm(x, w_1, bias=b_f, gelu=True, aux=pre, bn=bn, out=o)),
        ("fwd fc2", 2 * T * H * F, lambda bn, o=None: G.gemm(xf, w_2, bias=b_h, bn=bn, out=o)),
        ("dgrad fc2", 2 * T * F * H, lambda bn, o=None: G.gemm(dy_h, w_2.t(), bn=bn, out=o)),
        ("dgrad fc1", 2 * T * H * F, lambda bn, o=None: G.gemm(dy_f, w_1.t(), bn=bn, out=o)),
        ("dgrad out", 2 * T * H * H, lambda bn, o=None: G.gemm(dy_h, w_o.t(), bn=bn, out=o)),
        ("dgrad qkv", 2 * T * H * Q, lambda bn, o=None: G.gemm(dy_q, w_qkv.t(), bn=bn, out=o)),
        ("wgrad qkv", 2 * T * H * Q, lambda bn, o=None: G.gemm(x.t(), dy_q, out=g_qkv, accumulate=True, bn=bn)),
        ("wgrad out", 2 * T * H * H, lambda bn, o=None: G.gemm(x.t(), dy_h, out=g_o, accumulate=True, bn=bn)),
        ("wgrad fc1", 2 * T * H * F, lambda bn, o=None: G.gemm(x.t(), dy_f, out=g_1, accumulate=True, bn=bn)),
        ("wgrad fc2", 2 * T * F * H, lambda bn, o=None: G.gemm(xf.t(), dy_h, out=g_2, accumulate=True, bn=bn)),
    ]
    only = set(sys.argv[3].split(",")) if len(sys.argv) > 3 else None
    tot = {v: 0.0 for v in variants}
    for name, fl, f in cases:
        if only and name.split()[0] not in only:
            continue
        ok = ""
        if not name.startswith("wgrad"):
            ref = f(1).float()
            for v in variants:
                if v in (0, 1):
                    continue
                got = f(v).float()
                err = ((got - ref).abs().max() / ref.abs().max()).item()
                ok += f" err[{v}]={err:.1e}"
                if not err < 2e-2:
                    print(f"{name}: variant {v} WRONG (rel err {err})", flush=True)
        else:
            for v in [v for v in variants if v]:  # accumulate twice from zero: 2 x product
                out = {"wgrad qkv": g_qkv, "wgrad out": g_o, "wgrad fc1": g_1, "wgrad fc2": g_2}[name]
                out.zero_()
                f(v)
                f(v)
                r = out.float().clone()
                if v == [v for v in variants if v][0]:
                    ref = r
                else:
                    err = ((r - ref).abs().max() / ref.abs().max()).item()
                    ok += f" err[{v}]={err:.1e}"
                    if not err < 2e-2:
                        print(f"{name}: variant {v} WRONG (rel err {err})", flush=True)
        line = []
        for v in variants:
            fn = blas[name] if v == 0 else (lambda: f(v))
            t = min(timed(fn, iters) for _ in range(3))
            tot[v] += t
            line.append(f"{'blas' if v == 0 else f'bn{v}'} {t:7.1f}us {fl / t / 1e6:5.0f}TF")
        print(f"{name:14s} " + " | ".join(line) + ok, flush=True)
    print("layer total: " + ", ".join(f"bn{v} {t:.0f} us" for v, t in tot.items()), flush=True)


if __name__ == "__main__":
    main()
