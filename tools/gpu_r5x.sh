#!/bin/bash
# round 5: ping-pong split-K (1x1-conv weight gradients): exactness, per-shape A/B, ResNet-50 end to end
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6 step ppsk_test 300 python -u -m pytest tests/test_gemm_pp_splitk_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider && \
TAIL=12 step ppsk_bench 300 python -u tools/bench_wgrad_1x1.py && \
TAIL=5 step resnet 600 python bench.py --skip-gpt 1 --resnet-steps 10
