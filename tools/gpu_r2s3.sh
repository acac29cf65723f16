#!/bin/bash
# session-3 check: full GPU suite (incl. the native backward engine and reference-format program tests)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
