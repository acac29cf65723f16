"""LLaMA-2 decode serving throughput on one MI355X: random-init bf16 weights, batch B prompts of P tokens,
G greedy tokens each; eager per-step decode vs the hipGraph-captured decode step.
Usage: python tools/bench_serving.py [model=llama2-7b] [B=32] [P=512] [G=128]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "llama2-7b"
    B, P, G = (int(v) for v in (sys.argv[2:5] if len(sys.argv) > 4 else (32, 512, 128)))
    cfg = {"llama2-7b": LlamaConfig.llama2_7b, "llama2-13b": LlamaConfig.llama2_13b,
           "tiny": LlamaConfig.tiny}[name](max_position_embeddings=P + G + 64)
    paddle.set_device("gpu")
    paddle.set_default_dtype("bfloat16")
    paddle.seed(0)
    model = LlamaForCausalLM(cfg)
    paddle.set_default_dtype("float32")
    model.eval()
    ids = paddle.Tensor(torch.randint(0, cfg.vocab_size, (B, P), device="cuda"))
    for use_graph in (False, True, False, True):
        model.generate(ids, max_new_tokens=4, eos_token_id=-1, use_graph=use_graph)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model.generate(ids, max_new_tokens=1, eos_token_id=-1, use_graph=False)
        torch.cuda.synchronize()
        t_pref = time.perf_counter() - t0
        t0 = time.perf_counter()
        out, _ = model.generate(ids, max_new_tokens=G, eos_token_id=-1, use_graph=use_graph)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0 - t_pref
        tps = B * (G - 1) / dt
        print(f"{name} B={B} prompt={P} gen={G} {'hipGraph' if use_graph else 'eager   '}: "
              f"prefill {t_pref * 1e3:.1f} ms, decode {dt / (G - 1) * 1e3:.2f} ms/token, {tps:.0f} tokens/s",
              flush=True)


if __name__ == "__main__":
    main()
