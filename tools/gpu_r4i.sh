#!/bin/bash
# Round 4 box 9: the GPU test suite (fusion determinism, layout autotune with the fusion off), then ResNet-50 with
# the hoisted-constant BN apply kernels, fusion on and off.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15 step pytest_gpu_all 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
TAIL=3 step rn_on 400 python bench.py --skip-gpt 1 --resnet-steps 10 --steps 1 --warmup 3
TAIL=3 step rn_off 400 env FLAGS_conv_bn_fusion=0 python bench.py --skip-gpt 1 --resnet-steps 10 --steps 1 --warmup 3
