#!/bin/bash
# Round 4 box 8: the whole GPU test suite, then ResNet-50 with the conv -> BN fusion (narrow 1x1 statistics GEMM).
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15 step pytest_gpu_all 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
TAIL=5 step rn_fused2 400 python bench.py --skip-gpt 1 --resnet-steps 10 --steps 1 --warmup 3
