#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
step moe_tests 300 python -u -m pytest tests/test_moe_grouped.py tests/test_sharding_offload_gpu.py -x -v --timeout 120 --timeout-method thread
step moe_bench 300 python -u tools/bench_moe.py
