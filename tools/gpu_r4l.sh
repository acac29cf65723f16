#!/bin/bash
# Round 4 box 12: convolution weight-gradient tests after the slab-reduce rewrite, ResNet-50, then the GPT-3 13B
# small-op attribution (torch.profiler with call sites, one step outside the timed region).
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6 step pytest_conv 600 python -u -m pytest tests/test_conv_nhwc_gpu.py tests/test_production_geometry_gpu.py tests/test_conv3d_ndhwc_gpu.py tests/test_conv1d_nlc_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider
TAIL=3 step rn_slab 400 python bench.py --skip-gpt 1 --resnet-steps 10 --steps 1 --warmup 3
TAIL=60 step smallops 600 python tools/profile_small_ops.py
