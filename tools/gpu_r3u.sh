#!/bin/bash
# Per-direction conv + skinny GEMM tests, skinny GEMM timings, ResNet-50 bench with the per-direction choice.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12
export PADDLE_AMD_TUNING_FILE=$PWD/gpurun_out/tuning_overlay_resnet.json
step pytest_conv 300 python -u -m pytest tests/test_gemm.py -k skinny tests/test_conv_nhwc_gpu.py tests/test_bn_fused.py -m gpu -q -x --timeout 120 --timeout-method thread
step skinny 300 python tools/bench_skinny.py
step resnet 600 python bench.py --skip-gpt 1 --resnet-steps 10
