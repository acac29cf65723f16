#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step test_gemm 300 python -u -m pytest tests/test_gemm.py tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread
TAIL=10 step gemm_epi 300 python tools/bench_epi.py
TAIL=20 step gemm_variants 600 python tools/bench_mygemm.py 4096
