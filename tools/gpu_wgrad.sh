#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=9
step pytest_conv 300 python -u -m pytest tests/test_gemm.py -x -q -k "conv" --timeout 120 --timeout-method thread
step bench_wgrad 300 python -u tools/bench_wgrad.py
step resnet 900 python bench.py --skip-gpt 1 --resnet-steps 20
