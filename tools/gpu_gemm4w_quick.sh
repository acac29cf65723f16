#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=5 step gemm_abl 240 python tools/bench_gemm_abl.py
TAIL=20 step gemm_variants 480 python tools/bench_mygemm.py 4096
