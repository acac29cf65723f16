#!/bin/bash
# round-6 final: GPU test suite, smoke(), default bench (13B headline + ResNet-50 secondary) on the final tree
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
step final_pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider --maxfail 10
step final_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
TAIL=12
step final_bench 1000 python -u bench.py
