#!/bin/bash
# flash-attention numerics + microbench (+ kernel-only timing of the backward)
source "$(dirname "$0")/gpu_steps.sh"
step pytest_fa 600 python -m pytest tests/test_flash_attn.py tests/test_main_grad_fusion.py -m gpu -x -q
step bench_attn 600 python tools/bench_attn.py
step abl_fa 300 python tools/abl_fa.py
