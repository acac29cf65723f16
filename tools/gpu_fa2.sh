#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6
step pytest_fa 300 python -u -m pytest tests/test_flash_attn.py -x -q --timeout 120 --timeout-method thread
step abl_fa 300 python tools/abl_fa.py
