#!/bin/bash
# End-of-round-4 refresh of the secondary BASELINE configs: GPT-3 1.3B dygraph, LLaMA-2 7B (static auto-parallel
# engine = the 70B config's path, and fleet dygraph), LLaMA-2 7B serving decode.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step gpt1p3b_r4 600 python bench.py --model gpt3-1.3b --sharding-stage 0 --micro-batch 16 --accum 2 --resnet 0 --steps 5 --warmup 2
step llama7b_static_r4 900 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 2 --warmup 1 --resnet 0
step llama7b_fleet_r4 900 python bench.py --model llama2-7b --llama-engine fleet --micro-batch 2 --accum 4 --seq-len 4096 --steps 2 --warmup 1 --resnet 0
