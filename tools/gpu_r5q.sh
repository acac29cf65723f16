#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3 step gpt1p3b 400 python bench.py --model gpt3-1.3b --micro-batch 16 --accum 2 --steps 3 --warmup 2 --resnet 0
TAIL=3 step resnet 400 python bench.py --skip-gpt 1 --resnet 1
