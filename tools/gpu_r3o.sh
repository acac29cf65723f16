#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
export HIP_LAUNCH_BLOCKING=1
TAIL=4 step mfma16_check 60 ./tools/diag/mfma16_check
TAIL=8 step fa16_diag32 60 python -u tools/fa16_diag.py 32
TAIL=8 step fa16_diag300 60 python -u tools/fa16_diag.py 300
