#!/bin/bash
# remaining GPU tests (from the static/jit tests on) + GPT-13B micro-batch 4 x accum 4 (same global batch)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15 step pytest_gpu2 600 python -u -m pytest tests/test_static_jit.py tests/test_sync_bn_gpu.py tests/test_tensor_api.py tests/test_vision.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_mb4 900 python bench.py --micro-batch 4 --accum 4 --resnet 0
