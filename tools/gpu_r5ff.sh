#!/bin/bash
# GPT-3 1.3B (BASELINE secondary config): fused LM head + CE A/B, same box
source "$(dirname "$0")/gpu_steps.sh"
B="python bench.py --model gpt3-1.3b --sharding-stage 0 --micro-batch 16 --accum 2 --resnet 0 --steps 5 --warmup 2"
TAIL=1 step g13_base 600 $B && \
TAIL=1 step g13_fce 600 $B --fused-head-ce 1 && \
TAIL=1 step g13_base2 600 $B && \
TAIL=1 step g13_fce2 600 $B --fused-head-ce 1
grep -h "\[gpt\] loss" gpurun_out/g13_*.log
