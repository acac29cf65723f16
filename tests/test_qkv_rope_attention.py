"""qkv_rope_attention: fused projection output -> RoPE(q, k) -> causal attention, with the qkv gradient as one
buffer. GPU numerics against the fp32 composition (split + rotate + math attention); the CPU case checks the
composition path against the same reference."""
import pytest
import torch

from paddlepaddle_amd import ops
from paddlepaddle_amd.ops import _loader as L
from paddlepaddle_amd.ops.attention import attention_reference
from paddlepaddle_amd.ops.rope import _rotate_ref, rope_tables


def _reference(t, cos, sin, H, Hkv, D, neox):
    B, S, _ = t.shape
    tf = t.float()
    q, k, v = tf.split([H * D, Hkv * D, Hkv * D], -1)
    q = _rotate_ref(q.reshape(B, S, H, D), cos, sin, neox, False)
    k = _rotate_ref(k.reshape(B, S, Hkv, D), cos, sin, neox, False)
    return attention_reference(q, k, v.reshape(B, S, Hkv, D), causal=True)


def _check(dev, dt, B, S, H, Hkv, D, neox, tol):
    torch.manual_seed(0)
    t = (torch.randn(B, S, (H + 2 * Hkv) * D, device=dev) * 0.5).to(dt).requires_grad_(True)
    cos, sin = rope_tables(S, D, device=dev, neox=neox)
    o = ops.qkv_rope_attention(t, cos, sin, H, Hkv, D, neox=neox)
    tr = t.detach().float().requires_grad_(True)
    orf = _reference(tr, cos, sin, H, Hkv, D, neox)
    torch.testing.assert_close(o.float(), orf, atol=tol, rtol=tol)
    g = torch.randn_like(orf)
    o.backward(g.to(dt))
    orf.backward(g)
    torch.testing.assert_close(t.grad.float(), tr.grad, atol=tol * 2, rtol=tol * 2)
    return o


def test_qkv_rope_attention_cpu_composition():
    _check("cpu", torch.float32, 2, 32, 4, 2, 64, True, 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("H,Hkv,D,neox", [(8, 2, 128, True), (4, 4, 64, True), (4, 1, 128, False),
                                          (2, 2, 256, True)])
def test_qkv_rope_attention_hip(H, Hkv, D, neox):
    L.CALLS.pop("attn_aten_fallback", None)
    o = _check("cuda", torch.bfloat16, 2, 256, H, Hkv, D, neox, 3e-2)
    assert type(o.grad_fn).__name__ == "_QKVRopeAttnHIPBackward"
    assert L.CALLS.get("attn_aten_fallback", 0) == 0
    assert L.has("pa_rope_rows")
