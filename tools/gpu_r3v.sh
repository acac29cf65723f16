#!/bin/bash
# Skinny implicit 3x3 conv: tests, timings, ResNet-50 bench (re-times the 56x56 3x3 forward / data-grad keys).
source "$(dirname "$0")/gpu_steps.sh"
TAIL=14
export PADDLE_AMD_TUNING_FILE=$PWD/gpurun_out/tuning_overlay_resnet2.json
step pytest_conv 300 python -u -m pytest tests/test_conv_nhwc_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread
step skinny 300 python tools/bench_skinny.py
step resnet 600 python bench.py --skip-gpt 1 --resnet-steps 10
