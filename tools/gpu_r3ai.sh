#!/bin/bash
# halo conv: 32-pixel segments x 6 waves (PA_SKCONV_HALO=2) vs the default 16 x 12; conv tests under both.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
step halo12 120 python tools/bench_skinny.py sweep
PA_SKCONV_HALO=2 step halo2 120 python tools/bench_skinny.py sweep
PA_SKCONV_HALO=2 step pytest_conv2 300 python -u -m pytest tests/test_conv_nhwc_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k 3x3
step pytest_conv 300 python -u -m pytest tests/test_conv_nhwc_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread
