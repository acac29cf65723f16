#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step b13 900 python bench.py --resnet 0 --steps 2 --warmup 1
