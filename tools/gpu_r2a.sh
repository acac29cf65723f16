#!/bin/bash
# Round-2 first GPU pass: GPU tests + default bench (GPT-3 13B sharding-3 + ResNet-50) at the current tree.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_default 900 python bench.py
