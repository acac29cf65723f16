#!/bin/bash
# round 5: 70B PP4xTP2 stage proxy on the static engine (fused grads + fused clip), then the default bench
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3 step llama70b_stage 600 python bench.py --model llama2-70b-stage --micro-batch 1 --accum 4 --seq-len 4096 --steps 2 --warmup 1 --resnet 0 && \
TAIL=4 step bench_default 900 python bench.py
