#!/bin/bash
# halo conv: 8 vs 12 waves per workgroup.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
step pytest_conv 300 python -u -m pytest tests/test_conv_nhwc_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k 3x3
step halo8 120 python tools/bench_skinny.py sweep
PA_SKCONV_HALO=12 step halo12 120 python tools/bench_skinny.py sweep
PA_SKCONV_HALO=12 step pytest_conv12 300 python -u -m pytest tests/test_conv_nhwc_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k 3x3
