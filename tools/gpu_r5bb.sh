#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step llama_gpu 400 python -u -m pytest tests/test_llama.py tests/test_production_geometry_gpu.py tests/test_recompute_granularity.py tests/test_fused_grad_accumulation_gpu.py tests/test_serving_ops.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider && \
TAIL=2 step llama_fleet 300 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0 --llama-engine fleet
grep -h "\[llama\]" gpurun_out/llama_fleet.log
