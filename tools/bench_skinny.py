"""Memory-bound 1x1-convolution GEMMs of ResNet-50's 56x56 / 28x28 stages (batch 256): every hand-written
kernel variant (ops/gemm.py bn codes) against hipBLASLt (torch.mm), with the HBM roofline bytes.
Usage: python tools/bench_skinny.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlepaddle_amd.ops import gemm as G  # noqa: E402


def timeit(f, iters=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1000)
    return best


def main():
    P56, P28 = 256 * 56 * 56, 256 * 28 * 28
    cases = [  # (name, M, K, N, B K-major)
        ("fwd 64->64", P56, 64, 64, True), ("fwd 256->64", P56, 256, 64, True), ("fwd 64->256", P56, 64, 256, True),
        ("dgrad 64->64", P56, 64, 64, False), ("dgrad c1 (K64 N256)", P56, 64, 256, False),
        ("dgrad c3 (K256 N64)", P56, 256, 64, False), ("fwd 28 512->128", P28, 512, 128, True),
        ("dgrad 28 (K128 N512)", P28, 128, 512, False),
    ]
    for name, M, K, N, bk in cases:
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(N, K, device="cuda").bfloat16().t() if bk else torch.randn(K, N, device="cuda").bfloat16()
        byt = 2 * (M * K + M * N + K * N)
        line = f"{name:22s} M{M} K{K} N{N}: roofline@6TB/s {byt / 6e6:6.1f} us |"
        line += f" mm {timeit(lambda: torch.mm(a, b)):6.1f}"
        if G.skinny_supported(a, b):
            line += f" skinny {timeit(lambda: G.gemm_skinny(a, b)):6.1f}"
        for bn in (1, 256, 128, 160):
            try:
                t = timeit(lambda: G.gemm(a, b, bn=bn))
                line += f" bn{bn} {t:6.1f}"
            except Exception as e:  # noqa: BLE001
                line += f" bn{bn} err({type(e).__name__})"
        print(line, flush=True)


def conv3x3():
    from paddlepaddle_amd.ops import conv as C
    for (H, Cc, s) in [(56, 64, 1), (56, 64, 2)]:
        x = torch.randn(256, H, H, Cc, device="cuda").bfloat16()
        w = (torch.randn(Cc, Cc, 3, 3, device="cuda") * 0.05).bfloat16()
        wk = w.permute(0, 2, 3, 1).contiguous()
        t_sk = timeit(lambda: C._skinny_conv(x, wk, None, 256, H, H, Cc, Cc, 3, 3, s, 1))
        if s == 1:
            dy = torch.randn(256, H, H, Cc, device="cuda").bfloat16()
            t_wsk = timeit(lambda: C._skinny_wgrad(x, dy, w))
            t_wim = timeit(lambda: C._implicit_wgrad(x, dy, w, 256, H, H, Cc, Cc, 3, 3, 1, 1, 1, H, H))
            t_wmi = timeit(lambda: C._mi_bwd(x, w, dy, 1, 1, 1, [False, True]))
            ref = C._mi_bwd(x, w, dy, 1, 1, 1, [False, True])[1].float()
            err = (C._skinny_wgrad(x, dy, w).float() - ref).abs().max().item() / ref.abs().max().item()
            print(f"wgrad3x3 H{H} C{Cc}: skinny {t_wsk:6.1f} us | implicit {t_wim:6.1f} | MIOpen {t_wmi:6.1f} | "
                  f"rel err {err:.3g}", flush=True)
        if len(sys.argv) > 1:  # one PA_SKCONV_CFG per process (the launcher reads it once)
            print(f"cfg {os.environ.get('PA_SKCONV_CFG', '0')} H{H} s{s}: {t_sk:.1f} us", flush=True)
            continue
        t_im = timeit(lambda: C._implicit_fwd(x, wk, None, 256, H, H, Cc, Cc, 3, 3, s, 1, 1))
        t_mi = timeit(lambda: C._mi_fwd(x, w, None, s, 1, 1))
        ref = C._mi_fwd(x, w, None, s, 1, 1).float()
        err = (C._skinny_conv(x, wk, None, 256, H, H, Cc, Cc, 3, 3, s, 1).float() - ref).abs().max().item()
        fl = 2 * ref.numel() * Cc * 9
        print(f"conv3x3 H{H} C{Cc} s{s}: skinny {t_sk:6.1f} us ({fl / t_sk / 1e6:5.0f} TF) | implicit {t_im:6.1f} | "
              f"MIOpen {t_mi:6.1f} | max err {err:.3g} (max |y| {ref.abs().max().item():.3g})", flush=True)


if __name__ == "__main__":
    conv3x3()
    if len(sys.argv) > 1:
        sys.exit(0)
    main()
