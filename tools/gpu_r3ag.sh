#!/bin/bash
# swizzled 3x3 weight-gradient tiles: tests + timings + ResNet-50 bench (decisions kept in the overlay).
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6
export PADDLE_AMD_TUNING_FILE=$PWD/gpurun_out/tuning_overlay_resnet7.json
step pytest_wg 300 python -u -m pytest tests/test_conv_nhwc_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread
step skinny 200 python tools/bench_skinny.py sweep
step resnet 600 python bench.py --skip-gpt 1 --resnet-steps 10
step resnet_again 600 python bench.py --skip-gpt 1 --resnet-steps 10
