#!/bin/bash
# hand-written GEMM variants vs hipBLASLt on the GPT-3 13B shapes (+ square reference points)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step test_gemm 300 python -u -m pytest tests/test_gemm.py -x -q --timeout 120 --timeout-method thread
TAIL=4 step gemm_sq4k 300 python tools/bench_mygemm.py 4096 square
TAIL=20 step gemm_variants 600 python tools/bench_mygemm.py 4096
