#!/bin/bash
# quick GPU check of the kernels touched last
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step test_quick 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread
