#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
step pytest_fa 600 python -m pytest tests/test_flash_attn.py -x -q
step bench_attn 600 python tools/bench_attn.py
