#!/bin/bash
# Round 4 box 11: BN kernel microbenchmark after the hoisted-constant apply rewrite, ResNet-50 fused kernel window.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=30 step bench_bn 300 python tools/bench_bn.py
bash tools/gpu_prof.sh rn_fused2 --skip-gpt 1 --resnet-steps 8 > gpurun_out/prof_rn_fused2.log 2>&1; echo "prof rc=$?"
f=$(find gpurun_out/prof_rn_fused2 -name "*kernel_trace.csv" | head -1)
python tools/prof_window.py --ms 150 --top 40 "$f" > gpurun_out/rn_fused2_window.md 2>&1
grep "step=" gpurun_out/prof_rn_fused2/bench.log; head -30 gpurun_out/rn_fused2_window.md
