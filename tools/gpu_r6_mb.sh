#!/bin/bash
# round-6: 13B micro-batch A/B (global batch 16 either way)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
step b13_mb4_acc4 400 python bench.py --micro-batch 4 --accum 4 --steps 4 --warmup 2 --resnet 0
step b13_mb2_acc8 400 python bench.py --micro-batch 2 --accum 8 --steps 4 --warmup 2 --resnet 0
step b13_mb4_acc4_b 400 python bench.py --micro-batch 4 --accum 4 --steps 4 --warmup 2 --resnet 0
