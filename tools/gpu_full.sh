#!/bin/bash
# full GPU test suite + default bench
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15 step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_default 900 python bench.py
