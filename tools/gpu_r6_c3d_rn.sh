#!/bin/bash
# round-6: 3-D conv data gradient test + ResNet-50 kernel profile (graph replay, 1 GPU)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
step c3d_gpu 300 python -u -m pytest tests/test_conv3d_ndhwc_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider
bash "$(dirname "$0")/gpu_prof.sh" resnet_r6 --skip-gpt 1 --resnet-steps 8
