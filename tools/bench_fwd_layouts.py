"""GPT-3 13B forward GEMMs: torch.mm vs addmm (bias epilogue) vs transposed-weight layouts (hipBLASLt)."""
import torch


def t(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


M = 4096
for K, N in ((5120, 15360), (5120, 5120), (5120, 20480), (20480, 5120)):
    x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    w = torch.empty(K, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    wt = w.t().contiguous()
    b = torch.empty(N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    fl = 2 * M * N * K
    cands = {"mm(x,w)": lambda: torch.mm(x, w), "addmm(b,x,w)": lambda: torch.addmm(b, x, w),
             "mm(x,wt.t())": lambda: torch.mm(x, wt.t()), "addmm(b,x,wt.t())": lambda: torch.addmm(b, x, wt.t()),
             "mm+bias": lambda: torch.mm(x, w).add_(b),
             "gelu_epi(b,x,w)": lambda: torch._addmm_activation(b, x, w, use_gelu=True),
             "gelu_epi(b,x,wt.t())": lambda: torch._addmm_activation(b, x, wt.t(), use_gelu=True)}
    out = []
    for name, fn in cands.items():
        ms = min(t(fn), t(fn))
        out.append(f"{name} {fl / ms / 1e9:5.0f}")
    print(f"K={K} N={N}: " + " | ".join(out), flush=True)
