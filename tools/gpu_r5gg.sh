#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=1 step static_final 400 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0
grep -h "llama-static\]" gpurun_out/static_final.log
