#!/bin/bash
# round 3 check: full GPU suite, then the default bench (GPT-3 13B + ResNet-50)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=8 step bench_default 900 python bench.py
