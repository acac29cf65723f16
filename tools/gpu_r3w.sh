#!/bin/bash
# Skinny implicit 3x3 conv v2 (super-blocks, tap ring): tests + timings.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=14
step pytest_conv 300 python -u -m pytest tests/test_conv_nhwc_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread
step skinny 300 python tools/bench_skinny.py
