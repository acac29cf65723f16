#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step rc_gran 300 python -u -m pytest tests/test_recompute_granularity.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider
