#!/bin/bash
# round 3: 13B micro-batch A/B at the same global batch (mb2 x 8 vs mb4 x 4), back to back on one box
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3 step bench_13b_mb2 700 python bench.py --resnet 0 --steps 3 --warmup 1
TAIL=3 step bench_13b_mb4 700 python bench.py --resnet 0 --steps 3 --warmup 1 --micro-batch 4 --accum 4
TAIL=3 step bench_13b_mb2_again 700 python bench.py --resnet 0 --steps 3 --warmup 1
