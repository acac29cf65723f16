#!/bin/bash
# Skinny conv launch-config sweep, producer/sink tests, ResNet-50 bench.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=14
export PADDLE_AMD_TUNING_FILE=$PWD/gpurun_out/tuning_overlay_resnet3.json
step pytest_conv 300 python -u -m pytest tests/test_conv_nhwc_gpu.py tests/test_bn_fused.py -m gpu -q -x --timeout 120 --timeout-method thread
for c in 0 1 2 3; do PA_SKCONV_CFG=$c step skconv_cfg$c 120 python tools/bench_skinny.py sweep; done
step resnet 600 python bench.py --skip-gpt 1 --resnet-steps 10
