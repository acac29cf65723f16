#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=14
step pytest_fa 300 python -u -m pytest tests/test_flash_attn.py -x -q --timeout 120 --timeout-method thread
step bench_fa_fwd 300 python -u tools/bench_fa_fwd.py
