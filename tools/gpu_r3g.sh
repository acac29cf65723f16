#!/bin/bash
# round 3: BN / sink / captured-AdamW tests, whole GPU suite, default bench
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step new_tests 300 python -u -m pytest tests/test_bn_fused.py tests/test_train_step_graph.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=6 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=6 step bench_default 900 python bench.py
