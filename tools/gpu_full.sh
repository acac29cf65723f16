#!/bin/bash
# full GPU suite + smoke (what the driver runs at round end)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=25 step gpu_suite 1100 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider
TAIL=5 step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
