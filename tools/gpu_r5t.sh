#!/bin/bash
# round 5: static engine fused gradient accumulation — GPU parity test, then LLaMA-2 7B static vs fleet on one box
source "$(dirname "$0")/gpu_steps.sh"
B="python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 4 --warmup 1 --resnet 0"
TAIL=8 step engine_gpu_test 300 python -u -m pytest tests/test_static_engine_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider && \
TAIL=1 step static_c 300 $B && \
TAIL=1 step fleet_c 300 $B --llama-engine fleet && \
TAIL=1 step static_d 300 $B
grep -h "llama-static\]\|\[llama\]" gpurun_out/static_c.log gpurun_out/fleet_c.log gpurun_out/static_d.log
