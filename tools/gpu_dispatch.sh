#!/bin/bash
# native launch path: GPU tests + launch microbench + eager/graph decode A/B
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15 step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
TAIL=8 step launch 300 python -u tools/bench_launch.py
TAIL=6 step serving_native 600 python -u tools/bench_serving.py llama2-7b 32 512 128
PADDLE_AMD_CTYPES_LAUNCH=1 TAIL=6 step serving_ctypes 600 python -u tools/bench_serving.py llama2-7b 32 512 128
