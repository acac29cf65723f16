#!/bin/bash
# re-time every per-shape backend decision of the default bench (GPT-3 13B + ResNet-50), dump the table,
# install it in the box's tree and bench again with it
source "$(dirname "$0")/gpu_steps.sh"
export PADDLE_AMD_TUNING_FILE=$R/gpurun_out/overlay.json
TAIL=12 PADDLE_AMD_TUNING_RETUNE=1 PADDLE_AMD_TUNING_DUMP=$R/gpurun_out/gfx950.json step bench_tune 900 python bench.py
cp "$R/gpurun_out/gfx950.json" "$R/paddlepaddle_amd/ops/tuning/gfx950.json"
rm -f "$R/gpurun_out/overlay.json"
TAIL=12 step bench_tuned 900 python bench.py
