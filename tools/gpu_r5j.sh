#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
B="python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0"
TAIL=20 step multi_linear 300 python tools/bench_multi_linear.py
TAIL=2 step static_all_1f1b 300 $B
TAIL=2 step static_rms_1f1b 300 $B --static-passes rms_norm_residual
TAIL=2 step fleet_ref 300 $B --llama-engine fleet
