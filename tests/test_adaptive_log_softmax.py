"""nn.AdaptiveLogSoftmaxWithLoss / F.adaptive_log_softmax_with_loss (reference nn/functional/loss.py:4461): the
per-sample output equals the layer's full log_prob at the target, the loss is its negative mean, gradients flow."""
import numpy as np
import pytest

import paddlepaddle_amd as paddle


def test_adaptive_log_softmax_matches_log_prob_and_trains():
    paddle.seed(0)
    m = paddle.nn.AdaptiveLogSoftmaxWithLoss(16, 20, [5, 12], div_value=2.0, head_bias=True)
    x = paddle.randn([8, 16])
    y = paddle.to_tensor(np.array([0, 3, 5, 7, 11, 12, 19, 4]))
    out, loss = m(x, y)
    lp = m.log_prob(x).numpy()
    ref = lp[np.arange(8), y.numpy()]
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(float(loss), -ref.mean(), rtol=1e-5)
    np.testing.assert_allclose(np.exp(lp).sum(1), np.ones(8), rtol=1e-5)
    loss.backward()
    assert m.head_weight.grad is not None and m.tail_weights[1][1].grad is not None
    o1, l1 = m(x[0], y[0])                       # unbatched
    np.testing.assert_allclose(float(o1), ref[0], rtol=1e-5)
    with pytest.raises(ValueError):
        m(x, paddle.to_tensor(np.array([0, 1, 2, 3, 4, 5, 6, 20])))
