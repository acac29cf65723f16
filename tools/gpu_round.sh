#!/bin/bash
# One GPU call: GPU tests, default bench, rocprof of the GPT-13B step and of the ResNet-50 step.
source "$(dirname "$0")/gpu_steps.sh"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step bench_default 900 python bench.py
bash tools/gpu_prof.sh gpt13b_r1 --steps 2 --warmup 1 --resnet 0 || exit $?
bash tools/gpu_prof.sh resnet50_r1 --skip-gpt 1 --resnet-steps 10 || exit $?
