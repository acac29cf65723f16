#!/bin/bash
# Round 4 box 6: conv -> BN statistics fusion (kernel numerics, block parity), ResNet-50 A/B with the fusion on
# and off, then the production-geometry / layout-autotune GPU tests.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12 step pytest_convbn 300 python -u -m pytest tests/test_conv_bn_fusion_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread
TAIL=5 step rn_fused 500 python bench.py --skip-gpt 1 --resnet-steps 10 --steps 1 --warmup 3
TAIL=5 step rn_unfused 500 env FLAGS_conv_bn_fusion=0 python bench.py --skip-gpt 1 --resnet-steps 10 --steps 1 --warmup 3
TAIL=8 step pytest_prod 600 python -u -m pytest tests/test_production_geometry_gpu.py tests/test_layout_autotune.py -m gpu -x -q --timeout 300 --timeout-method thread
