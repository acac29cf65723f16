#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
step pytest_fa 600 python -m pytest tests/test_flash_attn.py -x -q
step bench_1p3b_norc 600 python bench.py --model gpt3-1.3b --micro-batch 8 --steps 4 --warmup 2 --recompute 0 --resnet 0
