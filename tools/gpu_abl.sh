#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
step abl_fa 300 python tools/abl_fa.py
