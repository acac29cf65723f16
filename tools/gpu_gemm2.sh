#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12
step pytest_gemm 300 python -u -m pytest tests/test_gemm.py tests/test_main_grad_fusion.py tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread
step bench13b 900 python bench.py --resnet 0
