#!/bin/bash
# default bench with the native allocator installed (compare with the caching-allocator run)
source "$(dirname "$0")/gpu_steps.sh"
PADDLE_AMD_ALLOCATOR=auto_growth TAIL=8 step bench_native_alloc 900 python bench.py
