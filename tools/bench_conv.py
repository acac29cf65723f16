"""ResNet-50 convolution shapes (batch 256, bf16, channels-last): MIOpen (torch conv2d) vs a plain
GEMM formulation for the 1x1 convolutions (hipBLASLt), forward / dgrad / wgrad, per layer.
Usage: python tools/bench_conv.py [batch]"""
import sys

import torch
import torch.nn.functional as F

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
SHAPES = [  # (name, Cin, Cout, k, stride, H_in, count per step)
    ("stem7x7", 3, 64, 7, 2, 224, 1),
    ("l1.c1a", 64, 64, 1, 1, 56, 1), ("l1.c1", 256, 64, 1, 1, 56, 2), ("l1.c2", 64, 64, 3, 1, 56, 3),
    ("l1.c3", 64, 256, 1, 1, 56, 3), ("l1.ds", 64, 256, 1, 1, 56, 1),
    ("l2.c1a", 256, 128, 1, 1, 56, 1), ("l2.c2a", 128, 128, 3, 2, 56, 1), ("l2.ds", 256, 512, 1, 2, 56, 1),
    ("l2.c1", 512, 128, 1, 1, 28, 3), ("l2.c2", 128, 128, 3, 1, 28, 3), ("l2.c3", 128, 512, 1, 1, 28, 4),
    ("l3.c1a", 512, 256, 1, 1, 28, 1), ("l3.c2a", 256, 256, 3, 2, 28, 1), ("l3.ds", 512, 1024, 1, 2, 28, 1),
    ("l3.c1", 1024, 256, 1, 1, 14, 5), ("l3.c2", 256, 256, 3, 1, 14, 5), ("l3.c3", 256, 1024, 1, 1, 14, 6),
    ("l4.c1a", 1024, 512, 1, 1, 14, 1), ("l4.c2a", 512, 512, 3, 2, 14, 1), ("l4.ds", 1024, 2048, 1, 2, 14, 1),
    ("l4.c1", 2048, 512, 1, 1, 7, 2), ("l4.c2", 512, 512, 3, 1, 7, 2), ("l4.c3", 512, 2048, 1, 1, 7, 3),
]


def timeit(f, iters=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000  # us


def main():
    tot = {"miopen": 0.0, "gemm": 0.0, "best": 0.0}
    for name, ci, co, k, s, H, cnt in SHAPES:
        pad = k // 2
        x = torch.randn(B, ci, H, H, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, k, k, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
        y = F.conv2d(x, w, None, s, pad)
        dy = torch.randn_like(y)
        Ho = y.shape[-1]
        flops = 2 * B * Ho * Ho * co * ci * k * k
        t_f = timeit(lambda: F.conv2d(x, w, None, s, pad))
        t_d = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [pad, pad], [1, 1], False,
                                                                 [0, 0], 1, [True, False, False]))
        t_w = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [pad, pad], [1, 1], False,
                                                                 [0, 0], 1, [False, True, False]))
        line = (f"{name:8s} {ci:4d}->{co:4d} k{k} s{s} H{H:3d}: miopen fwd {t_f:7.1f} dgrad {t_d:7.1f} "
                f"wgrad {t_w:7.1f} us ({3 * flops / (t_f + t_d + t_w) / 1e6:6.0f} TF)")
        m_tot = t_f + t_d + t_w
        best = m_tot
        if k == 1:
            xs = x[:, :, ::s, ::s] if s > 1 else x
            x2 = xs.permute(0, 2, 3, 1).reshape(-1, ci)  # NHWC rows (copy only when strided)
            w2 = w.view(co, ci)
            dy2 = dy.permute(0, 2, 3, 1).reshape(-1, co)
            g_f = timeit(lambda: x2 @ w2.t())
            g_d = timeit(lambda: dy2 @ w2)
            g_w = timeit(lambda: dy2.t() @ x2)
            line += f" | gemm fwd {g_f:7.1f} dgrad {g_d:7.1f} wgrad {g_w:7.1f} ({3 * flops / (g_f + g_d + g_w) / 1e6:6.0f} TF)"
            tot["gemm"] += cnt * (g_f + g_d + g_w)
            best = min(m_tot, g_f + g_d + g_w)
        else:
            tot["gemm"] += cnt * m_tot
        tot["miopen"] += cnt * m_tot
        tot["best"] += cnt * best
        print(line, flush=True)
    print(f"per-step conv total (x count): miopen {tot['miopen'] / 1000:.2f} ms, gemm-for-1x1 {tot['gemm'] / 1000:.2f} ms, "
          f"best-of {tot['best'] / 1000:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
