#!/bin/bash
# pairing: GPU tests, then the 13B bench with and without weight-gradient pairing
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6 step pair_tests 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_wgrad_pairing_gpu.py
TAIL=4 step bench_pair1 900 python bench.py --steps 3 --warmup 2 --resnet 0 --pair-wgrad 1
TAIL=4 step bench_pair0 900 python bench.py --steps 3 --warmup 2 --resnet 0 --pair-wgrad 0
