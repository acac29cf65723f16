"""Static auto-parallel engine on one MI355X: the engine registers its local linear / norm weights' gradients as
main grads, so the micro-batches' weight-gradient GEMMs accumulate into .grad in their epilogue (as fleet's
fuse_grad_accumulation). Training must match autograd accumulation (FLAGS_fused_grad_accumulation=0)."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle

pytestmark = pytest.mark.gpu


def _train(fused, steps=3):
    import paddlepaddle_amd.distributed as dist
    from paddlepaddle_amd.models.llama_auto import LlamaConfig, LlamaForCausalLMAuto, LlamaPretrainingCriterionAuto
    paddle.set_device("gpu:0")
    paddle.set_flags({"FLAGS_fused_grad_accumulation": fused})
    dist.auto_parallel.set_mesh(None)
    paddle.set_default_dtype("bfloat16")
    paddle.seed(11)
    cfg = LlamaConfig.tiny(num_hidden_layers=2, fuse_attention_qkv=True, fuse_attention_ffn=True)
    model, crit = LlamaForCausalLMAuto(cfg), LlamaPretrainingCriterionAuto(cfg)
    paddle.set_default_dtype("float32")
    opt = paddle.optimizer.AdamW(1e-3, parameters=model.parameters(), multi_precision=True)
    mesh = dist.ProcessMesh(np.arange(1).reshape(1, 1, 1), dim_names=["pp", "dp", "mp"])
    model, opt = dist.parallelize(model, opt, mesh, dp_config={"sharding_level": 0},
                                  mp_config={"parallelize_plan": {}}, pp_config={"split_spec": "layers"})
    st = dist.Strategy()
    st.pipeline.enable = True
    st.pipeline.accumulate_steps = 4
    dm = dist.to_static(model, None, crit, opt, st)
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, cfg.vocab_size, (8, 65), generator=g).cuda()
    x, y = paddle.Tensor(ids[:, :-1].contiguous()), paddle.Tensor(ids[:, 1:].contiguous())
    losses, ptrs = [], []
    for _ in range(steps):
        losses.append(float(dm(x, y)))
        eng = dm._engine
        ptrs.append(tuple(p._t.grad.data_ptr() for p in eng.local_params.values() if p._t.grad is not None))
    return losses, getattr(dm._engine, "fused_grads", 0), ptrs


def test_static_engine_fused_grad_accumulation_matches_autograd():
    try:
        fused, n, ptrs = _train(True)
        assert n >= 10, n  # linear / norm weights of the two layers
        assert len(set(ptrs)) == 1  # the same gradient storage every step
        ref, n0, _ = _train(False)
        assert n0 == 0
        np.testing.assert_allclose(fused, ref, rtol=2e-2, atol=2e-2)
    finally:
        paddle.set_flags({"FLAGS_fused_grad_accumulation": True})
