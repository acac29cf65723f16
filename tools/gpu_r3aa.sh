#!/bin/bash
# FA 16-key backward numerics, conv weight-grad re-timing (cold) via the ResNet bench, GPT bench with PA_FA_BWD16.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
export PADDLE_AMD_TUNING_FILE=$PWD/gpurun_out/tuning_overlay_resnet5.json
step pytest_fa16 200 python -u -m pytest tests/test_flash_attn.py -m gpu -q --timeout 120 --timeout-method thread -k bwd16
step resnet 600 python bench.py --skip-gpt 1 --resnet-steps 10
step resnet_again 600 python bench.py --skip-gpt 1 --resnet-steps 10
