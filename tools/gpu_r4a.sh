#!/bin/bash
# Round 4, first box: GPU test suite on the ADVICE fixes, GEMM harness reconciliation across operand
# distributions (tools/bench_gemm_dvfs.py), short 13B bench.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step gemm_dvfs 420 python -u tools/bench_gemm_dvfs.py
TAIL=12 step bench13b 600 python bench.py --steps 3 --warmup 2 --resnet 0
