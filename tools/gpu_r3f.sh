#!/bin/bash
# round 3: new GPU tests first (residual-grad sink, captured AdamW), whole suite, then ResNet-50 alone
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step new_tests 300 python -u -m pytest tests/test_bn_fused.py tests/test_train_step_graph.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=6 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=4 step bench_resnet 600 python bench.py --skip-gpt 1 --resnet-steps 20
