#!/bin/bash
# Refresh the secondary BASELINE configs on the current tree: GPT-3 1.3B dygraph, LLaMA-2 7B.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step gpt1p3b_mb16 600 python bench.py --model gpt3-1.3b --sharding-stage 0 --micro-batch 16 --accum 2 --resnet 0 --steps 5 --warmup 2
step llama7b 900 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 2 --warmup 1 --resnet 0
