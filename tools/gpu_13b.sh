#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step b13_mb4_rc1 700 python bench.py --model gpt3-13b --micro-batch 4 --steps 3 --warmup 1 --recompute 1 --resnet 0
step b13_mb2_rc0 700 python bench.py --model gpt3-13b --micro-batch 2 --steps 3 --warmup 1 --recompute 0 --resnet 0
