#!/bin/bash
# BASELINE config "GPT-3 1.3B dygraph bf16 on one MI355X": plain dygraph (no sharding), seq 2048
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4 step gpt1p3b_mb8 600 python bench.py --model gpt3-1.3b --sharding-stage 0 --micro-batch 8 --accum 4 --resnet 0 --steps 5 --warmup 2
TAIL=4 step gpt1p3b_mb16 600 python bench.py --model gpt3-1.3b --sharding-stage 0 --micro-batch 16 --accum 2 --resnet 0 --steps 5 --warmup 2
