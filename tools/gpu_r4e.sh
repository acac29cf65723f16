#!/bin/bash
# Round 4 box 5: production-geometry GPU tests, layout autotune parity, GPT-3 13B kernel profile (small-kernel census).
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
step pytest_prod 900 python -u -m pytest tests/test_production_geometry_gpu.py tests/test_layout_autotune.py -m gpu -x -q --timeout 300 --timeout-method thread
bash tools/gpu_prof.sh gpt13b_r4 --steps 2 --warmup 1 --resnet 0 > gpurun_out/prof_gpt13b_r4.log 2>&1; echo "prof rc=$?"
python tools/prof_summary.py gpurun_out/prof_gpt13b_r4 --top 60 > gpurun_out/gpt13b_r4_summary.md 2>&1; head -80 gpurun_out/gpt13b_r4_summary.md
