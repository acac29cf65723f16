"""Vocab-sliced fused LM head + cross-entropy (ops/lm_head.py) against the plain fp32 torch reference
cross_entropy(h @ w.T, labels): per-token loss, dh and dw. GPU: bf16 HIP path (hand-written GEMMs + slice
CE kernels) at a GPT-sized vocabulary, and the peak memory of the step is below the materialised-logits
path by about the size of the logits and their gradient."""
import numpy as np
import pytest
import torch

from paddlepaddle_amd import ops


def _ref(h, w, labels, ignore_index):
    h = h.detach().float().requires_grad_(True)
    w = w.detach().float().requires_grad_(True)
    loss = torch.nn.functional.cross_entropy(h @ w.t(), labels, ignore_index=ignore_index, reduction="none")
    return loss, h, w


def _check(dev, dt, T, H, V, n_slices, tol):
    g = torch.Generator().manual_seed(0)
    h = (torch.randn(T, H, generator=g) * 0.5).to(dev, dt).requires_grad_(True)
    w = (torch.randn(V, H, generator=g) * 0.05).to(dev, dt).requires_grad_(True)
    labels = torch.randint(0, V, (T,), generator=g).to(dev)
    labels[::7] = -100
    dl = torch.rand(T, generator=g).to(dev)
    loss = ops.lm_head_cross_entropy(h, w, labels, -100, n_slices)
    loss.backward(dl)
    rl, rh, rw = _ref(h, w, labels, -100)
    rl.backward(dl.float())
    np.testing.assert_allclose(loss.float().cpu().detach().numpy(), rl.cpu().detach().numpy(), rtol=tol, atol=tol)
    for got, ref in ((h.grad, rh.grad), (w.grad, rw.grad)):
        err = (got.float() - ref).abs().max().item()
        assert err <= tol * max(ref.abs().max().item(), 1e-3), err


@pytest.mark.parametrize("n_slices", [1, 3])
def test_lm_head_ce_matches_reference_cpu(n_slices):
    _check("cpu", torch.float32, 48, 32, 1000, n_slices, 1e-4)


@pytest.mark.gpu
def test_lm_head_ce_bf16_gpu_matches_fp32_and_saves_memory():
    _check("cuda", torch.bfloat16, 1024, 1024, 50304, 4, 3e-2)
    T, H, V = 4096, 2048, 50304
    h = torch.randn(T, H, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
    w = (torch.randn(V, H, device="cuda", dtype=torch.bfloat16) * 0.02).requires_grad_(True)
    labels = torch.randint(0, V, (T,), device="cuda")

    def peak(fn):
        h.grad = w.grad = None
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        fn().mean().backward()
        torch.cuda.synchronize()
        return torch.cuda.max_memory_allocated() - base

    fused = peak(lambda: ops.lm_head_cross_entropy(h, w, labels, -100, 4))
    plain = peak(lambda: ops.softmax_cross_entropy(ops.linear_nt(h, w), labels))
    # the plain path holds the [T, V] logits and their gradient at its peak; the fused one a vocabulary slice of
    # each (plus dW, which both produce)
    logits_bytes = T * V * 2
    assert plain - fused > 0.8 * logits_bytes, (fused, plain, logits_bytes)
