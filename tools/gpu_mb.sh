#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step b13_mb4_acc4 900 python bench.py --resnet 0 --micro-batch 4 --accum 4
step b13_mb2_acc8 900 python bench.py --resnet 0 --micro-batch 2 --accum 8
