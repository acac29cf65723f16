"""ATen-level census of one GPT-3 13B-shaped training step (fewer layers) on the bench's sharding-3 engine.

Counts every ATen op the step dispatches (forward, backward on the autograd threads, optimizer) with the bytes of
its tensor outputs, so the framework's own small kernels (zero fills, copies, casts, scalar multiplies) can be traced
to the op that launched them. Hand-written kernels called through pybind do not show here: this lists what runs on
ATen. Usage: python tools/op_census.py [--layers 2] [--micro-batch 4] [--accum 4]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.n = collections.Counter()
        self.bytes = collections.Counter()
        self.shapes = collections.defaultdict(collections.Counter)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__) if hasattr(func, "overloadpacket") else str(func)
        outs = out if isinstance(out, (tuple, list)) else (out,)
        b = 0
        shp = None
        for o in outs:
            if isinstance(o, torch.Tensor) and o.device.type != "meta":
                b += o.numel() * o.element_size()
                shp = shp or (tuple(o.shape), str(o.dtype).replace("torch.", ""))
        self.n[name] += 1
        self.bytes[name] += b
        if shp is not None:
            self.shapes[name][shp] += 1
        return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--layers", type=int, default=2)
    p.add_argument("--micro-batch", type=int, default=4)
    p.add_argument("--accum", type=int, default=4)
    p.add_argument("--seq-len", type=int, default=2048)
    p.add_argument("--model", default="gpt3-13b")
    a = p.parse_args()
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    from paddlepaddle_amd.distributed.sharding import group_sharded_parallel
    mk = {"gpt3-13b": GPTConfig.gpt3_13b, "gpt3-1.3b": GPTConfig.gpt3_1_3b, "tiny": GPTConfig.tiny}[a.model]
    cfg = mk(max_position_embeddings=max(a.seq_len, 128), num_hidden_layers=a.layers)
    paddle.set_default_dtype("bfloat16")
    paddle.seed(1234)
    model = GPTForPretraining(cfg)
    crit = GPTPretrainingCriterion(cfg)
    paddle.set_default_dtype("float32")
    opt = paddle.optimizer.AdamW(learning_rate=1e-4, parameters=model.parameters(), weight_decay=0.01,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0), multi_precision=True,
                                 apply_decay_param_fun=lambda n: not ("norm" in n or n.endswith("b_0")))
    model, opt, _ = group_sharded_parallel(model, opt, level="p_g_os")
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    data = torch.randint(0, cfg.vocab_size, (a.accum, a.micro_batch, a.seq_len + 1), device=dev)
    ids = [paddle.Tensor(data[i, :, :-1]) for i in range(a.accum)]
    lbl = [paddle.Tensor(data[i, :, 1:]) for i in range(a.accum)]

    def step():
        for i in range(a.accum):
            loss = crit(model(ids[i]), lbl[i]) * (1.0 / a.accum)
            loss.backward()
        opt.step()
        opt.clear_grad()

    for _ in range(2):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    c = Census()
    with c:
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    print(f"model {a.model} layers {a.layers} mb {a.micro_batch} accum {a.accum} seq {a.seq_len}: "
          f"{sum(c.n.values())} ATen ops in one step")
    print(f"{'op':40s} {'calls':>7s} {'MB out':>10s}  top shapes")
    for name, n in sorted(c.n.items(), key=lambda kv: -c.bytes[kv[0]]):
        top = ", ".join(f"{s[0]}{s[1]}x{k}" for s, k in c.shapes[name].most_common(3))
        print(f"{name:40s} {n:7d} {c.bytes[name] / 2**20:10.1f}  {top}")


if __name__ == "__main__":
    main()
