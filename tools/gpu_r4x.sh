#!/bin/bash
# End-of-round-4 ResNet-50 kernel window (rocprofv3 kernel trace, last 150 ms)
source "$(dirname "$0")/gpu_steps.sh"
bash tools/gpu_prof.sh rn_final --skip-gpt 1 --resnet-steps 8 > gpurun_out/prof_rn_final.log 2>&1; echo "prof rc=$?"
f=$(find gpurun_out/prof_rn_final -name "*kernel_trace.csv" | head -1)
python tools/prof_window.py --ms 150 --top 40 "$f" > gpurun_out/rn_final_window.md 2>&1
grep "img/s\|backend per shape" gpurun_out/prof_rn_final/bench.log | tail -4; head -14 gpurun_out/rn_final_window.md
