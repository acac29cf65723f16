#!/bin/bash
# Round 4 box 13: full GPU suite, smoke, default bench (GPT-3 13B N=1 + ResNet-50 secondary)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4 step pytest_gpu_all 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider
TAIL=2 step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAIL=4 step bench_default 900 python bench.py
