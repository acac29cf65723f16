#!/bin/bash
# flash attention: GPU tests of every variant, then the variant microbenchmark
source "$(dirname "$0")/gpu_steps.sh"
TAIL=30 step pytest_fa 600 python -u -m pytest tests/test_flash_attn.py tests/test_flash_attn_ext.py -x -q --timeout 120 --timeout-method thread
TAIL=20 step bench_attn_ext 600 python tools/bench_attn_ext.py
TAIL=10 step bench_attn 300 python tools/bench_attn.py
