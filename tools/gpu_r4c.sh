#!/bin/bash
# Round 4 box 3: weight-only int8/int4 + LLM.int8 kernels (tests + decode microbench), native interpreter on the
# HIP kernels (GPT PIR through the Predictor), layout autotune parity, fused LM-head+CE A/B on the 13B step.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
step pytest_r4c 600 python -u -m pytest tests/test_weight_only_quant.py tests/test_native_interp_kernels.py tests/test_layout_autotune.py -m gpu -x -q --timeout 300 --timeout-method thread
TAIL=30 step bench_wo 400 python -u tools/bench_wo.py
TAIL=4 step bench13b_fused_ce 600 python bench.py --steps 3 --warmup 2 --resnet 0 --fused-head-ce 1
TAIL=4 step bench13b_default 600 python bench.py --steps 3 --warmup 2 --resnet 0
