#!/bin/bash
# round 3: FA backward ablations, then the whole GPU suite, then the default bench
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12 step fa_bwd_abl 300 python -u tools/bench_fa_bwd_abl.py
TAIL=15 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=8 step bench_default 900 python bench.py
