#!/bin/bash
# Session re-entry validation: GPU tests, smoke, default bench, then the 16-key FA backward diagnostics.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=10
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
step bench_default 900 python bench.py
step fa16_diag 90 python tools/fa16_diag.py 64
step fa_bwd16 180 python tools/bench_fa_bwd16.py
