#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6
step pytest_gemm 300 python -u -m pytest tests/test_gemm.py tests/test_bn_fused.py tests/test_vision.py -x -q --timeout 120 --timeout-method thread
step resnet 600 python bench.py --skip-gpt 1
