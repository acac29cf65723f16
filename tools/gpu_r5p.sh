#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
B="python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0 --llama-engine fleet"
TAIL=8 step fga_test 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_grad_accumulation_gpu.py tests/test_native_train_executor.py -m gpu
TAIL=1 step l7_fga1 300 $B
FLAGS_fused_grad_accumulation=0 TAIL=1 step l7_fga0 300 $B
TAIL=1 step l7_fga1b 300 $B
TAIL=2 step l70_layer 300 python tools/bench_llama70b_layer.py
