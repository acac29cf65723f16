#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step b13_s3_mb2_acc8 900 python bench.py --model gpt3-13b --micro-batch 2 --accum 8 --steps 3 --warmup 1 --recompute 0 --resnet 1
