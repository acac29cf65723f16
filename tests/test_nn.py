"""nn layers, functional ops, optimizers, lr schedulers, save/load (CPU)."""
import os

import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
import paddlepaddle_amd.nn.functional as F


def test_linear_layout_and_state_dict(tmp_path):
    l = paddle.nn.Linear(4, 3)
    assert l.weight.shape == [4, 3] and l.bias.shape == [3]
    x = paddle.randn([2, 4])
    np.testing.assert_allclose(l(x).numpy(), x.numpy() @ l.weight.numpy() + l.bias.numpy(), rtol=1e-5, atol=1e-6)
    sd = l.state_dict()
    assert list(sd.keys()) == ["weight", "bias"]
    p = tmp_path / "m.pdparams"
    paddle.save(sd, str(p))
    l2 = paddle.nn.Linear(4, 3)
    l2.set_state_dict(paddle.load(str(p)))
    np.testing.assert_allclose(l2.weight.numpy(), l.weight.numpy())


def test_sequential_and_sublayers():
    m = paddle.nn.Sequential(paddle.nn.Linear(4, 8), paddle.nn.ReLU(), paddle.nn.Linear(8, 2))
    assert len(m.parameters()) == 4
    names = [n for n, _ in m.named_parameters()]
    assert names == ["0.weight", "0.bias", "2.weight", "2.bias"]
    assert m(paddle.randn([3, 4])).shape == [3, 2]
    m.eval()
    assert not m[0].training


def test_conv_pool_bn_shapes():
    x = paddle.randn([2, 3, 16, 16])
    c = paddle.nn.Conv2D(3, 8, 3, padding=1)
    assert c.weight.shape == [8, 3, 3, 3]
    y = paddle.nn.MaxPool2D(2)(paddle.nn.BatchNorm2D(8)(c(x)))
    assert y.shape == [2, 8, 8, 8]
    xh = paddle.randn([2, 16, 16, 3])
    ch = paddle.nn.Conv2D(3, 8, 3, padding=1, data_format="NHWC")
    assert ch(xh).shape == [2, 16, 16, 8]
    assert F.conv2d(x, c.weight, padding="SAME").shape == [2, 8, 16, 16]
    assert F.adaptive_avg_pool2d(x, 1).shape == [2, 3, 1, 1]


def test_batchnorm_running_stats_paddle_momentum():
    bn = paddle.nn.BatchNorm1D(4, momentum=0.9)
    x = paddle.randn([64, 4]) * 3 + 2
    bn(x)
    m = x.numpy().mean(0)
    np.testing.assert_allclose(bn._mean.numpy(), 0.1 * m, rtol=1e-4, atol=1e-5)


def test_layernorm_and_rmsnorm_reference():
    x = paddle.randn([4, 16])
    ln = paddle.nn.LayerNorm(16)
    xn = x.numpy()
    ref = (xn - xn.mean(-1, keepdims=True)) / np.sqrt(xn.var(-1, keepdims=True) + 1e-5)
    np.testing.assert_allclose(ln(x).numpy(), ref, rtol=1e-4, atol=1e-5)
    rn = paddle.nn.RMSNorm(16)
    np.testing.assert_allclose(rn(x).numpy(), xn / np.sqrt((xn ** 2).mean(-1, keepdims=True) + 1e-6), rtol=1e-4,
                               atol=1e-5)


def test_cross_entropy_semantics():
    logits = paddle.randn([5, 7])
    label = paddle.to_tensor([0, 1, 2, 3, -100])
    l = F.cross_entropy(logits, label)
    ref = torch.nn.functional.cross_entropy(torch.tensor(logits.numpy()), torch.tensor(label.numpy()))
    np.testing.assert_allclose(l.numpy(), ref.numpy(), rtol=1e-5)
    l2 = F.cross_entropy(logits, label.unsqueeze(-1), reduction="none")
    assert l2.shape == [5, 1]
    soft = F.softmax(paddle.randn([5, 7]))
    assert F.cross_entropy(logits, soft, soft_label=True).shape == []
    w = paddle.rand([7])
    lw = F.cross_entropy(logits, label, weight=w)
    refw = torch.nn.functional.cross_entropy(torch.tensor(logits.numpy()), torch.tensor(label.numpy()),
                                             weight=torch.tensor(w.numpy()))
    np.testing.assert_allclose(lw.numpy(), refw.numpy(), rtol=1e-5)


def test_multihead_attention_and_transformer():
    mha = paddle.nn.MultiHeadAttention(16, 4)
    x = paddle.randn([2, 5, 16])
    assert mha(x).shape == [2, 5, 16]
    enc = paddle.nn.TransformerEncoder(paddle.nn.TransformerEncoderLayer(16, 4, 32), 2)
    assert enc(x).shape == [2, 5, 16]
    t = paddle.nn.Transformer(16, 4, 1, 1, 32)
    assert t(x, paddle.randn([2, 3, 16])).shape == [2, 3, 16]


def test_rnn_layers():
    lstm = paddle.nn.LSTM(8, 16, num_layers=2, direction="bidirect")
    out, (h, c) = lstm(paddle.randn([3, 5, 8]))
    assert out.shape == [3, 5, 32] and h.shape == [4, 3, 16]
    gru = paddle.nn.GRU(8, 16)
    out, h = gru(paddle.randn([3, 5, 8]))
    assert out.shape == [3, 5, 16]
    cell = paddle.nn.LSTMCell(8, 16)
    y, (h, c) = cell(paddle.randn([3, 8]))
    assert y.shape == [3, 16]


@pytest.mark.parametrize("opt_name", ["SGD", "Momentum", "Adam", "AdamW", "Adamax", "Adagrad", "Adadelta", "RMSProp",
                                      "Lamb", "NAdam", "RAdam"])
def test_optimizers_decrease_loss(opt_name):
    paddle.seed(0)
    m = paddle.nn.Linear(8, 1)
    x = paddle.randn([64, 8])
    y = x.sum(axis=1, keepdim=True)
    lr = {"SGD": 0.05, "Momentum": 0.02, "Adadelta": 1.0, "Adagrad": 0.1}.get(opt_name, 0.02)
    opt = getattr(paddle.optimizer, opt_name)(learning_rate=lr, parameters=m.parameters())
    l0 = None
    for _ in range(60):
        loss = F.mse_loss(m(x), y)
        if l0 is None:
            l0 = float(loss)
        loss.backward()
        opt.step()
        opt.clear_grad()
    assert float(loss) < l0 * 0.7, (opt_name, l0, float(loss))


def test_adamw_matches_torch_reference():
    paddle.seed(1)
    m = paddle.nn.Linear(6, 3)
    ref = [p._t.detach().clone().requires_grad_(True) for p in m.parameters()]
    opt = paddle.optimizer.AdamW(0.01, parameters=m.parameters(), weight_decay=0.05)
    topt = torch.optim.AdamW(ref, lr=0.01, weight_decay=0.05)
    for _ in range(5):
        gs = [torch.randn_like(r) for r in ref]
        for p, g in zip(m.parameters(), gs):
            p._t.grad = g.clone()
        for r, g in zip(ref, gs):
            r.grad = g.clone()
        opt.step()
        topt.step()
    for p, r in zip(m.parameters(), ref):
        np.testing.assert_allclose(p.numpy(), r.detach().numpy(), rtol=1e-5, atol=1e-6)


def test_optimizer_state_dict_roundtrip(tmp_path):
    m = paddle.nn.Linear(4, 4)
    opt = paddle.optimizer.Adam(0.1, parameters=m.parameters())
    m(paddle.randn([2, 4])).sum().backward()
    opt.step()
    sd = opt.state_dict()
    assert any(k.endswith("_moment1_0") for k in sd)
    paddle.save(sd, str(tmp_path / "o.pdopt"))
    opt2 = paddle.optimizer.Adam(0.1, parameters=m.parameters())
    opt2.set_state_dict(paddle.load(str(tmp_path / "o.pdopt")))
    k = next(k for k in sd if k.endswith("_moment1_0"))
    p = next(p for p in m.parameters() if k.startswith(p.name))
    np.testing.assert_allclose(opt2._accumulators["moment1"][id(p)].numpy(), sd[k].numpy())


def test_grad_clip_global_norm():
    m = paddle.nn.Linear(4, 4)
    clip = paddle.nn.ClipGradByGlobalNorm(0.1)
    opt = paddle.optimizer.SGD(1.0, parameters=m.parameters(), grad_clip=clip)
    (m(paddle.randn([8, 4])) * 100).sum().backward()
    before = [p.numpy().copy() for p in m.parameters()]
    opt.step()
    delta = np.sqrt(sum(((p.numpy() - b) ** 2).sum() for p, b in zip(m.parameters(), before)))
    assert abs(delta - 0.1) < 1e-4


def test_lr_schedulers():
    s = paddle.optimizer.lr.StepDecay(1.0, step_size=2, gamma=0.5)
    vals = []
    for _ in range(5):
        vals.append(s())
        s.step()
    assert vals == [1.0, 1.0, 0.5, 0.5, 0.25]
    w = paddle.optimizer.lr.LinearWarmup(0.1, 4, 0.0, 0.1)
    assert w() == 0.0
    c = paddle.optimizer.lr.CosineAnnealingDecay(1.0, T_max=10)
    for _ in range(10):
        c.step()
    assert c() < 1e-6
    oc = paddle.optimizer.lr.OneCycleLR(1.0, total_steps=100)
    assert abs(oc() - 0.04) < 1e-6


def test_amp_auto_cast_o1_white_list():
    l = paddle.nn.Linear(4, 4)
    with paddle.amp.auto_cast(dtype="bfloat16"):
        y = l(paddle.randn([2, 4]))
        z = F.softmax(y)
    assert y.dtype == paddle.bfloat16
    assert z.dtype == paddle.bfloat16 or z.dtype == paddle.float32


def test_amp_decorate_o2_and_scaler():
    m = paddle.nn.Sequential(paddle.nn.Linear(4, 4), paddle.nn.LayerNorm(4))
    opt = paddle.optimizer.AdamW(0.01, parameters=m.parameters())
    m, opt = paddle.amp.decorate(m, opt, level="O2", dtype="bfloat16")
    assert m[0].weight.dtype == paddle.bfloat16 and m[1].weight.dtype == paddle.float32
    scaler = paddle.amp.GradScaler(init_loss_scaling=1024)
    with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
        loss = m(paddle.randn([2, 4])).astype("float32").mean()
    scaler.scale(loss).backward()
    scaler.step(opt)
    scaler.update()
    assert opt._multi_precision


def test_lenet_mnist_shaped_training_converges():
    paddle.seed(3)
    net = paddle.vision.models.LeNet()
    x = paddle.randn([32, 1, 28, 28])
    y = paddle.randint(0, 10, [32, 1])
    opt = paddle.optimizer.Adam(1e-3, parameters=net.parameters())
    for i in range(40):
        loss = F.cross_entropy(net(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
    assert float(loss) < 0.5


def test_dataloader_batches():
    class DS(paddle.io.Dataset):
        def __len__(self):
            return 10

        def __getitem__(self, i):
            return np.full((3,), i, np.float32), np.array([i], np.int64)

    dl = paddle.io.DataLoader(DS(), batch_size=4, shuffle=False, drop_last=False)
    batches = list(dl)
    assert len(batches) == 3
    assert batches[0][0].shape == [4, 3] and batches[0][1].numpy().ravel().tolist() == [0, 1, 2, 3]
    assert batches[-1][0].shape == [2, 3]


def test_gpt_tiny_trains_with_recompute():
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    paddle.seed(0)
    cfg = GPTConfig.tiny(use_recompute=True)
    m = GPTForPretraining(cfg)
    crit = GPTPretrainingCriterion(cfg)
    opt = paddle.optimizer.AdamW(3e-3, parameters=m.parameters())
    ids = paddle.randint(0, cfg.vocab_size, [2, 33])
    losses = []
    for _ in range(15):
        loss = crit(m(ids[:, :-1]), ids[:, 1:])
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0] - 1.0


def test_max_pool_padding_forms():
    """paddle's int / flat / nested padding forms on both layouts, incl. asymmetric (explicit -inf pad)."""
    import numpy as np
    x = paddle.to_tensor(np.random.RandomState(3).randn(2, 3, 7, 6).astype("float32"))
    F = paddle.nn.functional
    ref = F.max_pool2d(x, 3, 2, 1)
    np.testing.assert_array_equal(F.max_pool2d(x, 3, 2, [1, 1, 1, 1]).numpy(), ref.numpy())
    np.testing.assert_array_equal(F.max_pool2d(x, 3, 2, [[0, 0], [0, 0], [1, 1], [1, 1]]).numpy(), ref.numpy())
    xh = x.transpose([0, 2, 3, 1])
    got = F.max_pool2d(xh, 3, 2, [[0, 0], [1, 1], [1, 1], [0, 0]], data_format="NHWC")
    np.testing.assert_array_equal(got.numpy(), ref.numpy().transpose(0, 2, 3, 1))
    asym = F.max_pool2d(x, 3, 2, [[0, 0], [0, 0], [0, 2], [1, 0]]).numpy()
    xp = np.pad(x.numpy(), ((0, 0), (0, 0), (0, 2), (1, 0)), constant_values=-np.inf)
    want = np.stack([[[[xp[b, c, i * 2:i * 2 + 3, j * 2:j * 2 + 3].max() for j in range((xp.shape[3] - 3) // 2 + 1)]
                       for i in range((xp.shape[2] - 3) // 2 + 1)] for c in range(3)] for b in range(2)])
    np.testing.assert_array_equal(asym, want)


def test_fused_linear_dx_hook_on_the_generic_path():
    import torch
    from paddlepaddle_amd.ops import linear as Lin
    x = torch.randn(4, 3, requires_grad=True)
    w = torch.randn(3, 5, requires_grad=True)
    seen = []
    y = Lin.fused_linear(x, w, None, dx_hook=lambda g: (seen.append(g.shape), g.mul_(3))[0] and None)
    y.sum().backward()
    assert seen == [torch.Size([4, 3])]
    torch.testing.assert_close(x.grad, 3 * torch.ones(4, 5) @ w.detach().t())
