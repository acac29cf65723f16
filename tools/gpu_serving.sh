#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6
step pytest_llama 300 python -u -m pytest tests/test_llama.py tests/test_decode_attn.py -x -q --timeout 120 --timeout-method thread
step serving 600 python -u tools/bench_serving.py llama2-7b 32 512 128
