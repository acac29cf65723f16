#!/bin/bash
# Round 4 final profile: GPT-3 13B kernel summary on the end-of-round tree
source "$(dirname "$0")/gpu_steps.sh"
bash tools/gpu_prof.sh gpt13b_r4final --steps 2 --warmup 1 --resnet 0 > gpurun_out/prof_gpt13b_r4final.log 2>&1; echo "prof rc=$?"
python tools/prof_summary.py gpurun_out/prof_gpt13b_r4final --top 60 > gpurun_out/gpt13b_r4final_summary.md 2>&1; head -40 gpurun_out/gpt13b_r4final_summary.md
