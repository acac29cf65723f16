#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step llama7b 900 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 2 --warmup 1
step gpt13 900 python bench.py --resnet 0
