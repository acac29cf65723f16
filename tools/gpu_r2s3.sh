#!/bin/bash
# session-3 check: full GPU suite (incl. the native backward engine and reference-format program tests)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_mb4 600 python bench.py --resnet 0 --steps 3 --warmup 2 --micro-batch 4 --accum 4
