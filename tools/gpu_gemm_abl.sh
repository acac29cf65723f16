#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=5 step gemm_abl 300 python tools/bench_gemm_abl.py
