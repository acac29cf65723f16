#!/bin/bash
# Round 5 box 1: per-shape GEMM baseline of one 13B layer x micro-batch, then the default bench
source "$(dirname "$0")/gpu_steps.sh"
TAIL=16 step step_gemms 300 python tools/bench_step_gemms.py 20
TAIL=4 step bench_default 900 python bench.py
