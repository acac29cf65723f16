#!/bin/bash
# 3x3 weight-gradient halo kernel: tests + timings + ResNet-50 bench (convw keys of that shape re-timed).
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
export PADDLE_AMD_TUNING_FILE=$PWD/gpurun_out/tuning_overlay_resnet6.json
step pytest_wg 300 timeout -k 10 200 python -u -m pytest tests/test_conv_nhwc_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k wgrad_3x3
step skinny 200 python tools/bench_skinny.py sweep
step resnet 600 python bench.py --skip-gpt 1 --resnet-steps 10
