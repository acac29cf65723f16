#!/bin/bash
# round 3: new kernels / ops first (fp8 GEMM, serving, fused head), fp8 microbench, then GPT-13B with and
# without the fused vocab-sliced LM head + CE
source "$(dirname "$0")/gpu_steps.sh"
TAIL=20
step new_tests 400 python -u -m pytest tests/test_fp8_gemm.py tests/test_serving_ops.py tests/test_lm_head_ce.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=8 step bench_fp8 300 python -u tools/bench_fp8.py
TAIL=3 step bench_13b_plain 600 python bench.py --resnet 0 --steps 6 --warmup 2
TAIL=3 step bench_13b_fusedhead 600 python bench.py --resnet 0 --steps 6 --warmup 2 --fused-head-ce 1
