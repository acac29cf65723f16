#!/bin/bash
# vector main-grad fusion: GPU tests + GPT-3 13B bench
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_gpt 600 python bench.py --resnet 0
