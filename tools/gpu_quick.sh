#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6 step test_quick 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread
TAIL=4 step bench_gpt 900 python bench.py --resnet 0
