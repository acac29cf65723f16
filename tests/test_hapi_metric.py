"""hapi Model / callbacks / summary / flops and paddle.metric.
Reference test strategy: test/legacy_test/test_model.py, test_metrics.py, test_callbacks.py.
Metric parity is checked against scikit-learn (independent implementation)."""
import numpy as np
import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd.io import Dataset
from paddlepaddle_amd.static import InputSpec


def test_accuracy_metric_topk():
    rng = np.random.RandomState(0)
    logits = rng.randn(50, 7).astype("float32")
    labels = rng.randint(0, 7, (50, 1))
    m = paddle.metric.Accuracy(topk=(1, 3))
    c = m.compute(paddle.to_tensor(logits), paddle.to_tensor(labels))
    m.update(c)
    top = np.argsort(-logits, 1)
    exp1 = (top[:, :1] == labels).any(1).mean()
    exp3 = (top[:, :3] == labels).any(1).mean()
    np.testing.assert_allclose(m.accumulate(), [exp1, exp3], rtol=1e-6)
    assert m.name() == ["acc_top1", "acc_top3"]
    acc = paddle.metric.accuracy(paddle.to_tensor(logits), paddle.to_tensor(labels), k=3)
    np.testing.assert_allclose(float(acc), exp3, rtol=1e-6)


def test_precision_recall_auc_match_sklearn():
    sk = pytest.importorskip("sklearn.metrics")
    rng = np.random.RandomState(1)
    prob = rng.rand(400).astype("float32")
    lab = (rng.rand(400) < 0.3 + 0.5 * prob).astype("int64")
    p, r = paddle.metric.Precision(), paddle.metric.Recall()
    for i in range(0, 400, 100):
        p.update(prob[i:i + 100], lab[i:i + 100])
        r.update(prob[i:i + 100], lab[i:i + 100])
    pred = np.rint(prob).astype("int64")
    np.testing.assert_allclose(p.accumulate(), sk.precision_score(lab, pred), rtol=1e-6)
    np.testing.assert_allclose(r.accumulate(), sk.recall_score(lab, pred), rtol=1e-6)
    auc = paddle.metric.Auc()
    auc.update(np.stack([1 - prob, prob], 1), lab.reshape(-1, 1))
    np.testing.assert_allclose(auc.accumulate(), sk.roc_auc_score(lab, prob), atol=2e-3)


class _DS(Dataset):
    def __init__(self, n, seed=0):
        r = np.random.RandomState(seed)
        self.x = r.randn(n, 8).astype("float32")
        self.y = (self.x[:, 0] + self.x[:, 1] > 0).astype("int64").reshape(-1, 1)

    def __getitem__(self, i):
        return self.x[i], self.y[i]

    def __len__(self):
        return len(self.x)


def _model():
    paddle.seed(0)
    net = paddle.nn.Sequential(paddle.nn.Linear(8, 32), paddle.nn.ReLU(), paddle.nn.Linear(32, 2))
    m = paddle.Model(net, InputSpec([None, 8], "float32", "x"), InputSpec([None, 1], "int64", "y"))
    m.prepare(paddle.optimizer.Adam(1e-2, parameters=m.parameters()), paddle.nn.CrossEntropyLoss(),
              paddle.metric.Accuracy())
    return m


def test_model_fit_evaluate_predict_save_load(tmp_path):
    m = _model()
    before = m.evaluate(_DS(128, 1), batch_size=32, verbose=0)
    m.fit(_DS(512), _DS(128, 1), batch_size=32, epochs=4, verbose=0)
    after = m.evaluate(_DS(128, 1), batch_size=32, verbose=0)
    assert after["acc"] > 0.9 and after["loss"][0] < before["loss"][0]
    out = m.predict(_DS(20, 2), batch_size=8, stack_outputs=True)
    assert out[0].shape == (20, 2)
    m.save(str(tmp_path / "ck"))
    m2 = _model()
    m2.load(str(tmp_path / "ck"))
    np.testing.assert_array_equal(m2.predict(_DS(20, 2), batch_size=8, stack_outputs=True)[0], out[0])
    # inference export through jit.save
    m.save(str(tmp_path / "inf"), training=False)
    tl = paddle.jit.load(str(tmp_path / "inf"))
    np.testing.assert_allclose(tl(paddle.to_tensor(_DS(20, 2).x)).numpy(), out[0], rtol=1e-5, atol=1e-6)


def test_early_stopping_and_accumulation():
    m = _model()
    es = paddle.callbacks.EarlyStopping(monitor="acc", mode="max", patience=0, verbose=0, save_best_model=False)
    m.fit(_DS(256), _DS(64, 1), batch_size=32, epochs=50, verbose=0, callbacks=[es], accumulate_grad_batches=2)
    assert m.stop_training  # stopped well before 50 epochs once accuracy saturates


def test_summary_and_flops_lenet():
    net = paddle.vision.models.LeNet()
    info = paddle.summary(net, (1, 1, 28, 28))
    assert info["total_params"] == 61610 and info["trainable_params"] == 61610
    # MACs: conv1 6*28*28*(1*9+1) + conv2 16*10*10*(6*25+1) + fc 400*120 + 120*84 + 84*10, plus relu/pool
    fl = paddle.flops(net, [1, 1, 28, 28])
    convfc = 6 * 28 * 28 * 10 + 16 * 10 * 10 * 151 + 400 * 120 + 120 * 84 + 84 * 10
    assert fl >= convfc and fl < convfc * 1.2
