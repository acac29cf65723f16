#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=16 step gemm_variants 400 python tools/bench_gemm_variants.py 20 1,3,0
