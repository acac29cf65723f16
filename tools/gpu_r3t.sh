#!/bin/bash
# GPU tests from the point of the last failure on, then the per-direction conv timings.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6
step pytest_gpu_pp 300 python -u -m pytest tests/test_pp_schedules.py -m gpu -x -q --timeout 120 --timeout-method thread
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step conv_dir 400 python tools/bench_conv_dir.py
