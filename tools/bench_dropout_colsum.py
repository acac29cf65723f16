"""Dropout backward + bias-gradient column sum at the GPT-3 13B out-proj / FFN2 shape ([4096, 5120] bf16):
unfused (pa_dropout_bwd, then pa_colsum = partial + fold kernels) vs fused (pa_dropout_bwd_colsum, then
pa_fold_partials)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from paddlepaddle_amd.ops import _loader as L  # noqa: E402


def timed(fn, iters=200):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    rows, cols = 4096, 5120
    dy = torch.randn(rows, cols, device="cuda").to(torch.bfloat16)
    dx = torch.empty_like(dy)
    db = torch.empty(cols, device="cuda", dtype=torch.bfloat16)
    ws = torch.empty(256 * cols, device="cuda", dtype=torch.float32)
    npart = int(L.lib().pa_colsum_nparts(rows))
    code = L.dcode(dy)

    def unfused():
        L.call("pa_dropout_bwd", L.ptr(dy), L.ptr(dx), dy.numel(), 0.1, 1234, code, L.stream_ptr())
        L.call("pa_colsum", L.ptr(dx), L.ptr(db), L.ptr(ws), rows, cols, code, L.stream_ptr())

    def fused():
        L.call("pa_dropout_bwd_colsum", L.ptr(dy), L.ptr(dx), L.ptr(ws), rows, cols, 0.1, 1234, code, L.stream_ptr())
        L.call("pa_fold_partials", L.ptr(ws), L.ptr(db), cols, npart, code, L.stream_ptr())

    unfused()
    ref_dx, ref_db = dx.clone(), db.float().clone()
    fused()
    assert torch.equal(ref_dx, dx)
    assert (db.float() - ref_db).abs().max().item() <= 0.05 * ref_db.abs().max().item()
    tu, tf = timed(unfused), timed(fused)
    print(f"dropout bwd + bias colsum [{rows}, {cols}] bf16: unfused {tu * 1e6:.1f} us, fused {tf * 1e6:.1f} us "
          f"(x{tu / tf:.2f})", flush=True)


if __name__ == "__main__":
    main()
