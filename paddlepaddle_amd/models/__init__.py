"""Model zoo used by the benchmarks (GPT-3, LLaMA, ResNet)."""
from .gpt import GPTConfig, GPTModel, GPTForPretraining, GPTPretrainingCriterion  # noqa: F401
from .llama import (LlamaConfig, LlamaModel, LlamaForCausalLM, LlamaPretrainingCriterion,  # noqa: F401
                    LlamaDecoderLayer)
