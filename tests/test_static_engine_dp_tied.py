"""Static auto-parallel engine, plain data parallelism with a weight that reaches the dp-split computation through
another op (a tied, transposed embedding table used as the LM head): its gradient is all-reduced inside autograd,
so it must stay out of the once-per-step flat-buffer synchronisation (else it comes out dp-degree times too
large). ZeRO on such a model raises. Also: an embedding with padding_idx on a vocabulary-sharded table keeps the
table-gather path (the vocab-parallel rewrite drops padding_idx). 2 gloo ranks vs single-process training."""
import numpy as np
import pytest
import torch

from test_distributed_cpu import _setup, _spawn

STEPS = 3


def _model(paddle, padding_idx=None):
    class Tied(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.emb = paddle.nn.Embedding(32, 16, padding_idx=padding_idx)
            self.fc = paddle.nn.Linear(16, 16)

        def forward(self, ids):
            h = paddle.tanh(self.fc(self.emb(ids)))
            return paddle.matmul(h, self.emb.weight, transpose_y=True)  # tied LM head
    return Tied()


class _CE:
    def __init__(self, paddle):
        self.paddle = paddle

    def __call__(self, logits, labels):
        return self.paddle.nn.functional.cross_entropy(logits.reshape([-1, 32]), labels.reshape([-1]))


def _data():
    g = torch.Generator().manual_seed(9)
    ids = torch.randint(0, 32, (8, 9), generator=g)
    ids[:, 3] = 0  # padding rows
    return ids


def _worker(rank, world, port, mode, q):
    paddle = _setup(rank, world, port)
    import paddlepaddle_amd.distributed as dist
    dist.auto_parallel.set_mesh(None)
    paddle.seed(3)
    model = _model(paddle, padding_idx=0 if mode == "pad_tp" else None)
    opt = paddle.optimizer.AdamW(0.05, parameters=model.parameters())
    strategy = dist.Strategy()
    if mode == "pad_tp":
        mesh = dist.ProcessMesh(np.arange(world).reshape(1, world), dim_names=["dp", "mp"])
        dist.shard_tensor(model.emb.weight, mesh, [dist.Replicate(), dist.Shard(0)])
    else:
        mesh = dist.ProcessMesh(np.arange(world).reshape(world, 1), dim_names=["dp", "mp"])
    dist.auto_parallel.set_mesh(mesh)
    dist.shard_layer(model, mesh)  # distributed (replicated) parameters: the static engine path
    if mode == "zero":
        strategy.sharding["enable"] = True
        strategy.sharding["degree"] = world
        strategy.sharding["stage"] = 1
        try:
            dm = dist.to_static(model, None, _CE(paddle), opt, strategy)
            ids = _data()
            dm(paddle.Tensor(ids[:, :-1]), paddle.Tensor(ids[:, 1:]))
            q.put((rank, "no error"))
        except NotImplementedError as e:
            q.put((rank, str(e)))
        paddle.distributed.barrier()
        return
    dm = dist.to_static(model, None, _CE(paddle), opt, strategy)
    ids = _data()
    losses = [float(dm(paddle.Tensor(ids[:, :-1]), paddle.Tensor(ids[:, 1:]))) for _ in range(STEPS)]
    eng = dm._engine
    q.put((rank, losses, len(eng._keep_ctp), eng.vocab_parallel_ops))
    paddle.distributed.barrier()


def _reference(padding_idx=None):
    import os
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    paddle.distributed.auto_parallel.set_mesh(None)
    paddle.seed(3)
    model = _model(paddle, padding_idx)
    opt = paddle.optimizer.AdamW(0.05, parameters=model.parameters())
    ids = _data()
    out = []
    for _ in range(STEPS):
        loss = _CE(paddle)(model(paddle.Tensor(ids[:, :-1])), paddle.Tensor(ids[:, 1:]))
        loss.backward()
        opt.step()
        opt.clear_grad()
        out.append(float(loss))
    return out


def test_dp2_tied_transposed_weight_matches_single_process():
    ref = _reference()
    for rank, losses, kept, _vp in _spawn(_worker, "dp", world=2):
        np.testing.assert_allclose(losses, ref, rtol=2e-5, atol=1e-6, err_msg=f"rank {rank}")
        assert kept == 1, kept  # the tied table keeps its in-autograd all-reduce


def test_zero_with_tied_weight_raises():
    for rank, msg in _spawn(_worker, "zero", world=2):
        assert "sharding off" in msg, msg


def test_vocab_sharded_embedding_with_padding_idx_keeps_gather_path():
    ref = _reference(padding_idx=0)
    for rank, losses, _kept, vp in _spawn(_worker, "pad_tp", world=2):
        np.testing.assert_allclose(losses, ref, rtol=2e-5, atol=1e-6, err_msg=f"rank {rank}")
        assert vp == 0, vp  # not rewritten into the vocab-parallel lookup
