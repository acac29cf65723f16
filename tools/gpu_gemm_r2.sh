#!/bin/bash
# hand-written GEMM variants vs hipBLASLt on the GPT-3 13B shapes
source "$(dirname "$0")/gpu_steps.sh"
TAIL=20 step gemm_variants 600 python tools/bench_mygemm.py 4096
