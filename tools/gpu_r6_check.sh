#!/bin/bash
# round-6 session check: GPU test suite, then the default bench
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
step pytest_gpu 780 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_default 360 python bench.py
