#!/bin/bash
# Full validation (GPU tests, smoke, default bench) + GPT-3 13B kernel trace.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
step bench_default 900 python bench.py
bash tools/gpu_prof.sh gpt13b_r3s2 --resnet 0 --steps 2 --warmup 1 > gpurun_out/prof_gpt.log 2>&1; echo "prof rc=$?"
