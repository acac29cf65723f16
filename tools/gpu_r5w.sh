#!/bin/bash
# round 5: fp8 ping-pong GEMM — exactness tests, then the microbench vs the generic kernel and hipBLASLt fp8
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step fp8_tests 300 python -u -m pytest tests/test_fp8_gemm.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider && \
TAIL=8 step fp8_bench 300 python -u tools/bench_fp8.py
