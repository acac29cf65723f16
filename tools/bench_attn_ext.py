"""Micro-benchmark of the HIP flash attention variants (TF/s of useful work, CUDA events) against ATen SDPA
(aotriton / math) on the same inputs: plain causal, dense bool padding mask, additive bias, flashmask documents,
dropout, GQA and a varlen batch."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from paddlepaddle_amd.ops.attention import attention  # noqa: E402


def timed(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it / 1e3


def fwd_bwd(fn, q, k, v, g):
    tf = timed(lambda: fn(q, k, v))
    tb = timed(lambda: torch.autograd.grad(fn(q, k, v), (q, k, v), g)) - tf
    return tf, tb


def run(name, B, S, H, Hk, D, flops_frac, ours, ref=None):
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hk, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hk, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    fl = 4 * B * H * S * S * D * flops_frac
    tf, tb = fwd_bwd(ours, q, k, v, g)
    line = f"{name:28s} B{B} S{S} H{H}/{Hk} D{D}: ours fwd {fl / tf / 1e12:5.0f} TF bwd {2.5 * fl / tb / 1e12:5.0f} TF"
    if ref is not None:
        rf, rb = fwd_bwd(ref, q, k, v, g)
        line += f" | sdpa fwd {fl / rf / 1e12:5.0f} TF bwd {2.5 * fl / rb / 1e12:5.0f} TF"
    print(line, flush=True)


def sdpa(mask=None, causal=False, p=0.0):
    def f(q, k, v):
        H, Hk = q.shape[2], k.shape[2]
        kt, vt = k.transpose(1, 2), v.transpose(1, 2)
        if H != Hk:
            kt, vt = kt.repeat_interleave(H // Hk, 1), vt.repeat_interleave(H // Hk, 1)
        return F.scaled_dot_product_attention(q.transpose(1, 2), kt, vt, attn_mask=mask, is_causal=causal,
                                              dropout_p=p).transpose(1, 2)
    return f


B, S, H, D = 2, 2048, 40, 128
run("causal", B, S, H, H, D, 0.5, lambda q, k, v: attention(q, k, v, causal=True), sdpa(causal=True))
lens = torch.tensor([1800, 1200], device="cuda")
pad = (torch.arange(S, device="cuda")[None, None, None] < lens[:, None, None, None])
run("bool padding mask [B,1,1,S]", B, S, H, H, D, 0.75, lambda q, k, v: attention(q, k, v, mask=pad),
    sdpa(mask=pad))
bias = (torch.randn(1, H, S, S, device="cuda") * 0.5).to(torch.bfloat16)
run("additive bf16 bias [1,H,S,S]", B, S, H, H, D, 1.0, lambda q, k, v: attention(q, k, v, mask=bias),
    sdpa(mask=bias))
lts = torch.empty(S, dtype=torch.int32)
for s0, n in ((0, 512), (512, 1024), (1536, 512)):
    lts[s0:s0 + n] = s0 + n
se = lts.view(1, 1, S, 1).expand(B, 1, S, 1).contiguous().cuda()
run("flashmask 3 documents", B, S, H, H, D, 0.5 * 0.6,
    lambda q, k, v: attention(q, k, v, causal=True, startend_row_indices=se))
run("causal + dropout 0.1", B, S, H, H, D, 0.5, lambda q, k, v: attention(q, k, v, causal=True, dropout=0.1),
    sdpa(causal=True, p=0.1))
run("GQA 64/8 causal", 1, 4096, 64, 8, 128, 0.5, lambda q, k, v: attention(q, k, v, causal=True),
    sdpa(causal=True))
# varlen: 8 sequences, 16k tokens
lens = [4096, 1024, 3000, 2048, 512, 2400, 1920, 1384]
cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
T_, Hh = int(cu[-1]), 32
q = torch.randn(T_, Hh, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
g = torch.randn_like(q)
fn = lambda: attention(q, q, q, causal=True, cu_seqlens_q=cu, cu_seqlens_k=cu, max_seqlen_q=max(lens),  # noqa: E731
                       max_seqlen_k=max(lens))
fl = sum(4 * Hh * n * n * 128 * 0.5 for n in lens)
tf = timed(fn)
tb = timed(lambda: torch.autograd.grad(fn(), q, g)) - tf
print(f"{'varlen causal 8 seqs':28s} {T_} tokens H{Hh} D128: ours fwd {fl / tf / 1e12:5.0f} TF bwd "
      f"{2.5 * fl / tb / 1e12:5.0f} TF", flush=True)
