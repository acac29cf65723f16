#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=16
step pytest_gemm 300 python -u -m pytest tests/test_gemm.py -x -q -k small_m --timeout 120 --timeout-method thread
step bench_smallm 300 python -u tools/bench_smallm.py
