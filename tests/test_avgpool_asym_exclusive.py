"""avg_pool2d with asymmetric padding and exclusive=True (the average over each window's real elements)."""
import numpy as np

import paddlepaddle_amd as paddle


def test_avg_pool2d_asymmetric_exclusive_matches_nanmean():
    a = np.random.RandomState(0).rand(2, 3, 6, 5).astype("float32")
    for pads, ceil in (([0, 1, 1, 0], False), ([1, 0, 0, 2], True)):
        y = paddle.nn.functional.avg_pool2d(paddle.to_tensor(a), 3, stride=2, padding=pads, exclusive=True,
                                            ceil_mode=ceil).numpy()
        pt, pb, pl, pr = pads
        ap = np.pad(a, ((0, 0), (0, 0), (pt, pb), (pl, pr)), constant_values=np.nan)
        H, W = ap.shape[2], ap.shape[3]
        rnd = (lambda v: -(-v // 2)) if ceil else (lambda v: v // 2)
        Ho, Wo = rnd(H - 3) + 1, rnd(W - 3) + 1
        ref = np.zeros((2, 3, Ho, Wo), "float32")
        for i in range(Ho):
            for j in range(Wo):
                ref[:, :, i, j] = np.nanmean(ap[:, :, 2 * i:2 * i + 3, 2 * j:2 * j + 3], axis=(2, 3))
        assert y.shape == ref.shape
        np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5)
