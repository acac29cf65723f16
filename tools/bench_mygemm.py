"""Hand-written MFMA GEMM vs hipBLASLt (torch.mm) on the GPT-3 13B linear shapes, all three products
(fwd x.W, dgrad dy.W^T, wgrad x^T.dy), same random bf16 data, interleaved rounds in one process."""
import sys

import torch

sys.path.insert(0, ".")
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


VARIANTS = {1: "pp-256", 2: "4w-agpr"}


def main():
    dt = torch.bfloat16
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    shapes = [(5120, 15360), (5120, 5120), (5120, 20480), (20480, 5120), (5120, 50304)]
    if len(sys.argv) > 2 and sys.argv[2] == "square":  # the guide's 4096^3 / 8192^3 reference points
        shapes = [(M, M)]
    for K, N in shapes:
        x = torch.empty(M, K, device="cuda", dtype=dt).uniform_(-1, 1)
        w = torch.empty(K, N, device="cuda", dtype=dt).uniform_(-1, 1)
        dy = torch.empty(M, N, device="cuda", dtype=dt).uniform_(-1, 1)
        cases = {
            "fwd": (lambda: torch.mm(x, w), lambda bn: G.gemm(x, w, bn=bn)),
            "dgrad": (lambda: torch.mm(dy, w.t()), lambda bn: G.gemm(dy, w.t(), bn=bn)),
            "wgrad": (lambda: torch.mm(x.t(), dy), lambda bn: G.gemm(x.t(), dy, bn=bn)),
        }
        fl = 2 * M * N * K
        for name, (ref, mine) in cases.items():
            rr = ref().float()
            errs = {bn: ((mine(bn).float() - rr).abs().max() / rr.abs().max()).item() for bn in VARIANTS}
            tr, tm = [], {bn: [] for bn in VARIANTS}
            for _ in range(3):
                tr.append(timeit(ref))
                for bn in VARIANTS:
                    tm[bn].append(timeit(lambda: mine(bn)))
            tr = min(tr)
            line = f"M={M} K={K} N={N} {name:5s}: hipBLASLt {fl / tr / 1e9:5.0f} TF ({tr:.3f} ms)"
            for bn in VARIANTS:
                t = min(tm[bn])
                line += f" | {VARIANTS[bn]} {fl / t / 1e9:5.0f} TF x{tr / t:.2f} err {errs[bn]:.0e}"
            print(line, flush=True)
        del x, w, dy


if __name__ == "__main__":
    main()
