#!/bin/bash
# Round 4 box 4: weight-only kernel v2 (column tiles by M) tests + decode microbench, layout-autotune stage diff.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6
step pytest_wo 600 python -u -m pytest tests/test_weight_only_quant.py -m gpu -x -q --timeout 300 --timeout-method thread
TAIL=30 step bench_wo2 400 python -u tools/bench_wo.py
TAIL=14 step diag_autotune 300 python -u tools/diag_autotune.py
