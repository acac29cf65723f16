#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=15 step graphs 300 python -u -m pytest tests/test_cuda_graphs.py tests/test_native_allocator.py tests/test_llama.py -x -v --timeout 200 --timeout-method thread -m gpu
