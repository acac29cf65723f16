#!/bin/bash
# measure the per-shape GEMM / conv backend choices for the bench models and dump them (committed table source)
source "$(dirname "$0")/gpu_steps.sh"
export PADDLE_AMD_TUNING_FILE=/tmp/tuning_overlay.json
PADDLE_AMD_TUNING_DUMP=gpurun_out/tuning_gpt_resnet.json step tune_bench 900 python bench.py --steps 2 --warmup 1
PADDLE_AMD_TUNING_DUMP=gpurun_out/tuning_llama.json step tune_llama 900 python bench.py --model llama2-7b --seq-len 4096 --accum 2 --steps 1 --warmup 1
step bench_tuned 600 python bench.py
