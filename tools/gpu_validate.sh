#!/bin/bash
# Validation pass: all GPU tests, smoke(), default bench. Stops at the first crash/timeout.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
step bench_default 900 python bench.py
