#!/bin/bash
# re-time every per-shape backend decision of the default bench (GPT-3 13B + ResNet-50) and dump the table
source "$(dirname "$0")/gpu_steps.sh"
export PADDLE_AMD_TUNING_FILE=$R/gpurun_out/overlay.json
TAIL=12 PADDLE_AMD_TUNING_DUMP=$R/gpurun_out/gfx950.json step bench_tune 900 python bench.py
TAIL=12 step bench_tuned 900 python bench.py
