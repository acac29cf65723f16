#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=14 step step_gemms 300 python tools/bench_step_gemms.py 20
TAIL=2 step gpt13b 400 python bench.py --resnet 0
TAIL=6 step seg_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_segmented_gemm_gpu.py tests/test_wgrad_pairing_gpu.py -m gpu
