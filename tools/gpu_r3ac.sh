#!/bin/bash
# LDS halo-tile 3x3 conv: tests, timings vs the gather kernel, ResNet-50 bench.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6
step pytest_conv 300 python -u -m pytest tests/test_conv_nhwc_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread
step halo 120 python tools/bench_skinny.py sweep
PA_SKCONV_HALO=0 step gather 120 python tools/bench_skinny.py sweep
step resnet 600 python bench.py --skip-gpt 1 --resnet-steps 10
