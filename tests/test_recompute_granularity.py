"""recompute_granularity (PaddleNLP: full / full_attn / core_attn) and no_recompute_layers on the GPT and LLaMA
models: the checkpointed scope changes (counted), losses and gradients do not."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
import importlib

R = importlib.import_module("paddlepaddle_amd.distributed.fleet.recompute")


def _grads(kind, gran=None, skip=()):
    paddle.seed(5)
    if kind == "llama":
        from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM
        cfg = LlamaConfig.tiny(num_hidden_layers=3)
        model = LlamaForCausalLM(cfg)
    else:
        from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining
        cfg = GPTConfig.tiny(num_hidden_layers=3, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        model = GPTForPretraining(cfg)
    cfg.use_recompute = gran is not None
    if gran is not None:
        cfg.recompute_granularity = gran
        cfg.no_recompute_layers = skip
    model.train()
    ids = torch.randint(0, cfg.vocab_size, (2, 17), generator=torch.Generator().manual_seed(1))
    logits = model(paddle.Tensor(ids[:, :-1]))
    loss = paddle.nn.functional.cross_entropy(logits.reshape([-1, cfg.vocab_size]), paddle.Tensor(ids[:, 1:]).reshape([-1]))
    loss.backward()
    return float(loss), {n: p.grad.numpy().copy() for n, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("kind", ["llama", "gpt"])
@pytest.mark.parametrize("gran,skip,calls", [("full", (), 3), ("full_attn", (), 3), ("core_attn", (), 3),
                                             ("full", (0, 2), 1), ("full_attn", (1,), 2)])
def test_recompute_granularity_keeps_gradients(kind, gran, skip, calls, monkeypatch):
    n = []
    orig = R.recompute

    def counting(fn, *a, **k):
        n.append(fn)
        return orig(fn, *a, **k)
    ref_loss, ref = _grads(kind)
    monkeypatch.setattr(R, "recompute", counting)
    loss, got = _grads(kind, gran, skip)
    assert len(n) == calls, (gran, skip, len(n))
    assert abs(loss - ref_loss) < 1e-6
    assert got.keys() == ref.keys()
    for k in ref:
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("gran", ["full", "full_attn", "core_attn"])
def test_recompute_granularity_llama_bf16_gpu(gran):
    """The HIP training path (fused qkv -> RoPE -> flash attention op, residual-fused RMSNorm, main-grad GEMMs):
    each granularity matches no recompute at the bf16 noise floor."""
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM

    def run(g):
        paddle.set_device("gpu:0")
        paddle.set_default_dtype("bfloat16")
        paddle.seed(5)
        cfg = LlamaConfig.tiny(num_hidden_layers=2)
        model = LlamaForCausalLM(cfg)
        paddle.set_default_dtype("float32")
        cfg.use_recompute = g is not None
        if g:
            cfg.recompute_granularity = g
        ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=torch.Generator().manual_seed(1)).cuda()
        logits = model(paddle.Tensor(ids[:, :-1]))
        loss = paddle.nn.functional.cross_entropy(logits.astype("float32").reshape([-1, cfg.vocab_size]),
                                                  paddle.Tensor(ids[:, 1:]).reshape([-1]))
        loss.backward()
        return float(loss), {n: p.grad._t.float().cpu().numpy() for n, p in model.named_parameters() if p.grad is not None}
    ref_loss, ref = run(None)
    loss, got = run(gran)
    assert abs(loss - ref_loss) < 1e-3
    for k in ref:
        scale = np.abs(ref[k]).max() + 1e-6
        assert np.abs(got[k] - ref[k]).max() <= 3e-2 * scale, k
