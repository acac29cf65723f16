#!/bin/bash
# Fused BN+ReLU(+add) / multi-tensor Momentum: GPU numerics, ResNet-50 bench, rocprof summary.
source "$(dirname "$0")/gpu_steps.sh"
step test_bn 600 python -m pytest tests/test_bn_fused.py tests/test_decode_attn.py tests/test_vision.py -x -q
step bench_resnet 600 python bench.py --skip-gpt 1 --resnet 1
bash tools/gpu_prof.sh resnet_fused --skip-gpt 1 --resnet 1 --resnet-steps 5 || exit $?
