#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
step pytest_dec 400 python -u -m pytest tests/test_gemm.py tests/test_fused_decode.py tests/test_llama.py tests/test_decode_attn.py -x -q -m gpu --timeout 120 --timeout-method thread
step serving 600 python -u tools/bench_serving.py
step smallm 300 python -u tools/bench_smallm.py
