#!/bin/bash
# round 3: new serving / fused-head tests first, then the whole GPU suite, then the default bench
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15
step new_tests 300 python -u -m pytest tests/test_serving_ops.py tests/test_lm_head_ce.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=8 step bench_default 900 python bench.py
