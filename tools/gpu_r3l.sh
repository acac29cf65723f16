#!/bin/bash
# round 3: depthwise conv kernels (tests + vs MIOpen), whole GPU suite and smoke under the native engine default
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4 step dwconv_tests 300 python -u -m pytest tests/test_dwconv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=10 step dwconv_bench 300 python -u tools/bench_dwconv.py
TAIL=6 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=3 step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
