#!/bin/bash
# full GPU test suite + default bench (GPT-3 13B + ResNet-50) + rocprof of the 13B step
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_default 900 python bench.py
