#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step wgrad_epi 300 python tools/bench_wgrad_epi.py
