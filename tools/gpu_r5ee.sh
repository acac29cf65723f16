#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3 step bench_default_graph 900 python bench.py
