#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=20
step blaslib 400 python -u tools/bench_blaslib.py
