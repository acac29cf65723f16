#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
B="python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0"
TAIL=1 step static_fused 300 $B
TAIL=1 step fleet_fused 300 $B --llama-engine fleet
TAIL=1 step static_unfused 300 $B --llama-fused-attn 0
TAIL=1 step static_fused2 300 $B
TAIL=3 step llama70b_stage 600 python bench.py --model llama2-70b-stage --micro-batch 1 --accum 4 --seq-len 4096 --steps 2 --warmup 1 --resnet 0
