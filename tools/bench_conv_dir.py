"""ResNet-50 convolutions (batch 256, bf16 NHWC) per direction: the hand-written paths (ops/conv.py: 1x1 as GEMMs,
KxK implicit GEMM forward / stride-1 data gradient / split-K weight gradient) against MIOpen's forward, data
gradient and weight gradient, each timed alone. Prints the per-step total of the whole-conv choice (what
ops/conv.py picked before per-direction choices) and of the per-direction best.
Usage: python tools/bench_conv_dir.py [batch]"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlepaddle_amd.ops import conv as C  # noqa: E402
from paddlepaddle_amd.ops import gemm as G  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
SHAPES = [  # (name, Cin, Cout, k, stride, H_in, count per step)
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
    best = 1e30
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1000)
    return best  # us


def main():
    tot_whole = tot_dir = tot_mi = 0.0
    for name, ci, co, k, s, H, cnt in SHAPES:
        pad = k // 2
        x = torch.randn(B, H, H, ci, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(co, ci, k, k, device="cuda") * 0.05).bfloat16()
        xc = x.permute(0, 3, 1, 2)
        wc = w.contiguous(memory_format=torch.channels_last)
        yc = F.conv2d(xc, wc, None, s, pad)
        dy = torch.randn(yc.permute(0, 2, 3, 1).shape, device="cuda", dtype=torch.bfloat16)
        dyc = dy.permute(0, 3, 1, 2)
        m = [timeit(lambda: F.conv2d(xc, wc, None, s, pad)),
             timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [s, s], [pad, pad], [1, 1], False,
                                                                [0, 0], 1, [True, False, False])),
             timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [s, s], [pad, pad], [1, 1], False,
                                                                [0, 0], 1, [False, True, False]))]
        o = [None, None, None]
        if k == 1:
            w2 = w.reshape(co, ci)

            def fwd():
                xs = x[:, ::s, ::s, :].contiguous() if s > 1 else x
                return G.gemm(xs.reshape(-1, ci), w2.t())
            dy2 = dy.reshape(-1, co)
            xs2 = (x[:, ::s, ::s, :].contiguous() if s > 1 else x).reshape(-1, ci)

            def dgrad():
                dx = G.gemm(dy2, w2)
                if s > 1:
                    full = torch.zeros(B, H, H, ci, dtype=dx.dtype, device=dx.device)
                    full[:, ::s, ::s, :] = dx.view(B, H // s, H // s, ci)
                return dx

            def wgrad():
                return G.gemm_splitk(dy2.t(), xs2, C._splits(co, ci, dy2.shape[0]))
            o = [timeit(fwd), timeit(dgrad), timeit(wgrad)]
        else:
            wk = w.permute(0, 2, 3, 1).contiguous()
            Ho = dy.shape[1]
            o[0] = timeit(lambda: C._implicit_fwd(x, wk, None, B, H, H, ci, co, k, k, s, pad, 1))
            if s == 1 and co % 64 == 0:
                wt = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()
                o[1] = timeit(lambda: C._implicit_fwd(dy, wt, None, B, Ho, Ho, co, ci, k, k, 1, k - 1 - pad, 1))
            o[2] = timeit(lambda: C._implicit_wgrad(x, dy, w, B, H, H, ci, co, k, k, s, pad, 1, Ho, Ho))
        own = [t if t is not None else float("inf") for t in o]
        own_whole = sum(a if a is not None else b for a, b in zip(o, m))  # MIOpen where ours has no path
        whole = min(sum(m), own_whole)
        per_dir = sum(min(a, b) for a, b in zip(own, m))
        tot_whole += cnt * whole
        tot_dir += cnt * per_dir
        tot_mi += cnt * sum(m)
        fmt = lambda t: "   --  " if t is None else f"{t:7.1f}"  # noqa: E731
        print(f"{name:7s} {ci:4d}->{co:4d} k{k} s{s} H{H:3d} | fwd ours {fmt(o[0])} mi {m[0]:7.1f} | dgrad ours "
              f"{fmt(o[1])} mi {m[1]:7.1f} | wgrad ours {fmt(o[2])} mi {m[2]:7.1f} | whole {whole:7.1f} "
              f"per-dir {per_dir:7.1f} us", flush=True)
    print(f"per step (x count): MIOpen only {tot_mi / 1000:.2f} ms, whole-conv choice {tot_whole / 1000:.2f} ms, "
          f"per-direction choice {tot_dir / 1000:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
