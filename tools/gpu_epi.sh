#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12 step test_pool 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q -k maxpool --timeout 120 --timeout-method thread
TAIL=10 step gemm_epi 300 python tools/bench_epi.py
