#!/bin/bash
# FA backward with conflict-free LDS swizzles: tests, timing, PMC
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3 step pytest_fa 400 python -u -m pytest tests/test_flash_attn.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=5 step fa_bwd16 200 python -u tools/bench_fa_bwd16.py
TAIL=3 step pmc_fa 300 bash tools/gpu_pmc_fa2.sh
