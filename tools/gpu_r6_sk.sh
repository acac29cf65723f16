#!/bin/bash
# round-6: split-K weight-gradient candidate (tests + GPT-3 1.3B, BASELINE config mb 16 x accum 2)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step sk_gpu 300 python -u -m pytest tests/test_gemm_pp_splitk_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider
export PADDLE_AMD_TUNING_DUMP="$R/gpurun_out/tune_1p3b_sk.json"
step g1_sk 300 python bench.py --model gpt3-1.3b --resnet 0 --steps 4 --warmup 2 --micro-batch 16 --accum 2
unset PADDLE_AMD_TUNING_DUMP
step g1_sk_b 300 python bench.py --model gpt3-1.3b --resnet 0 --steps 4 --warmup 2 --micro-batch 16 --accum 2
