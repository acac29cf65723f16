#!/bin/bash
# Conv per-direction choice with cold-cache timing + hipBLASLt 1x1 candidate: tests, ResNet-50 bench (decisions kept).
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
export PADDLE_AMD_TUNING_FILE=$PWD/gpurun_out/tuning_overlay_resnet4.json
step pytest_conv 300 python -u -m pytest tests/test_conv_nhwc_gpu.py tests/test_bn_fused.py -m gpu -q -x --timeout 120 --timeout-method thread
step resnet 600 python bench.py --skip-gpt 1 --resnet-steps 10
step resnet_again 600 python bench.py --skip-gpt 1 --resnet-steps 10
