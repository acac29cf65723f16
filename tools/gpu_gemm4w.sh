#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4 step gemm_sq4k 240 python tools/bench_mygemm.py 4096 square
TAIL=20 step gemm_variants 480 python tools/bench_mygemm.py 4096
