#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6 step seg_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_segmented_gemm_gpu.py tests/test_wgrad_pairing_gpu.py -m gpu
TAIL=16 step multi_linear 300 python tools/bench_multi_linear.py
TAIL=6 step wgrad_pair 200 python tools/bench_wgrad_epi.py pair
TAIL=2 step gpt13b_pair0 400 python bench.py --resnet 0
TAIL=2 step gpt13b_pair1 400 python bench.py --resnet 0 --pair-wgrad 1
