"""ops.ffn_gelu off the HIP path (CPU) is fc1 + tanh-GELU then fc2 (ops/linear.py); the GPT MLP routes through it."""
import torch


def test_ffn_gelu_cpu_matches_two_linears():
    from paddlepaddle_amd.ops import linear as LIN
    torch.manual_seed(0)
    x = torch.randn(3, 5, 16, requires_grad=True)
    w1, b1 = torch.randn(16, 32, requires_grad=True), torch.randn(32, requires_grad=True)
    w2, b2 = torch.randn(32, 8, requires_grad=True), torch.randn(8, requires_grad=True)
    y = LIN.ffn_gelu(x, w1, b1, w2, b2)
    ref = torch.nn.functional.gelu(x @ w1 + b1, approximate="tanh") @ w2 + b2
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
