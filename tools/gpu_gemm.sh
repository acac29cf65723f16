#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=40
step pytest_gemm 300 python -u -m pytest tests/test_gemm.py -x -q --timeout 120 --timeout-method thread
step bench_mygemm 300 python -u tools/bench_mygemm.py 4096
