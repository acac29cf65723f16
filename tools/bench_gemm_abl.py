"""Ablations of the 4-wave GEMM (timing only): full kernel vs no global loads / no fragment reads / no barrier,
plus the ping-pong kernel and hipBLASLt on the same shape (interleaved rounds, random data)."""
import sys

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    for (M, N, K) in [(4096, 20480, 5120), (8192, 8192, 8192)]:
        x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(K, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2 * M * N * K
        cands = {"hipblaslt": lambda: torch.mm(x, w), "pp": lambda: G.gemm(x, w, out=out, bn=1),
                 "4w": lambda: G.gemm(x, w, out=out, bn=2)}
        for abl in (0, 5, 6, 7, 8):
            cands[f"4w-abl{abl}"] = (lambda abl=abl: L.call("pa_gemm_bf16_4w_abl", L.ptr(x), L.ptr(w), L.ptr(out),
                                                              M, N, K, abl, L.stream_ptr()))
        t = {k: [] for k in cands}
        for _ in range(3):
            for k, fn in cands.items():
                t[k].append(timeit(fn))
        print(f"M={M} N={N} K={K}: " + " | ".join(f"{k} {fl / min(v) / 1e9:5.0f} TF" for k, v in t.items()), flush=True)


if __name__ == "__main__":
    main()
