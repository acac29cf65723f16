#!/bin/bash
# round 3: GPU suite again (after the lm-head memory assertion fix), then a kernel-trace profile of the 13B step
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
bash "$R/tools/gpu_prof.sh" gpt13b_r3 --resnet 0 --steps 2 --warmup 1
