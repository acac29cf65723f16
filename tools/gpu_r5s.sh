#!/bin/bash
# round 5: LLaMA-2 7B static engine (compiled per-node argument builders) vs fleet on one box
source "$(dirname "$0")/gpu_steps.sh"
B="python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 4 --warmup 1 --resnet 0"
TAIL=1 step static_a 300 $B && \
TAIL=1 step fleet_a 300 $B --llama-engine fleet && \
TAIL=1 step static_b 300 $B && \
TAIL=1 step fleet_b 300 $B --llama-engine fleet
