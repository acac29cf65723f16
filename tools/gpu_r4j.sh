#!/bin/bash
# Round 4 box 10: convolution kernels after the depth-dimension change (2-D production geometry, NHWC conv suite,
# 1-D NLC, 3-D NDHWC, conv -> BN fusion), then ResNet-50.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12 step pytest_conv 600 python -u -m pytest tests/test_conv_nhwc_gpu.py tests/test_production_geometry_gpu.py tests/test_conv1d_nlc_gpu.py tests/test_conv3d_ndhwc_gpu.py tests/test_conv_bn_fusion_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider
TAIL=3 step rn_after3d 400 python bench.py --skip-gpt 1 --resnet-steps 10 --steps 1 --warmup 3
