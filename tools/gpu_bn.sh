#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=30 step bench_bn 300 python tools/bench_bn.py
