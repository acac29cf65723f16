#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=5
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_attn 600 python tools/bench_attn.py
