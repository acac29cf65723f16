#!/bin/bash
# round-6: GPU suite + smoke after the last CPU-side fixes
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step final2_pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider --maxfail 10
step final2_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
