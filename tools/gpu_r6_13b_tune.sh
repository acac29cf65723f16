#!/bin/bash
# round-6: GEMM tuning decisions of the 13B mb4 default + GPT-3 1.3B micro-batch variants (global batch 32)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step nt_gpu 300 python -u -m pytest tests/test_native_train_executor.py tests/test_fusion_passes.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
export PADDLE_AMD_TUNING_DUMP="$R/gpurun_out/tune_13b_mb4.json"
step t13_mb4 400 python bench.py --resnet 0 --steps 2 --warmup 1
export PADDLE_AMD_TUNING_DUMP="$R/gpurun_out/tune_1p3b_mb16.json"
step g1_mb16 300 python bench.py --model gpt3-1.3b --resnet 0 --steps 4 --warmup 2 --micro-batch 16 --accum 2
export PADDLE_AMD_TUNING_DUMP="$R/gpurun_out/tune_1p3b_mb32.json"
step g1_mb32 300 python bench.py --model gpt3-1.3b --resnet 0 --steps 4 --warmup 2 --micro-batch 32 --accum 1
export PADDLE_AMD_TUNING_DUMP="$R/gpurun_out/tune_1p3b_mb8.json"
step g1_mb8 300 python bench.py --model gpt3-1.3b --resnet 0 --steps 4 --warmup 2 --micro-batch 8 --accum 4
unset PADDLE_AMD_TUNING_DUMP
step g1_mb16_b 300 python bench.py --model gpt3-1.3b --resnet 0 --steps 4 --warmup 2 --micro-batch 16 --accum 2
step l70_stage_acc8 600 python bench.py --model llama2-70b-stage --seq-len 4096 --micro-batch 1 --accum 8 --steps 2 --warmup 1 --resnet 0
