#!/bin/bash
# round-6: the whole GPU test suite (assertion failures do not stop it; a crash / timeout does)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
step pytest_gpu_all 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider --maxfail 10
