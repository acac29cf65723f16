#!/bin/bash
# GPU tests + 13B bench (+ rocprof) after the forward-weight layout cache.
source "$(dirname "$0")/gpu_steps.sh"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step bench_13b 900 python bench.py --resnet 0
bash tools/gpu_prof.sh gpt13b_wtcache --steps 2 --warmup 1 --resnet 0 || exit $?
