#!/bin/bash
# Round 4 box 7: conv -> BN fusion parity tests, then ResNet-50 kernel windows with the fusion on and off.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6 step pytest_convbn 300 python -u -m pytest tests/test_conv_bn_fusion_gpu.py tests/test_production_geometry_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
bash tools/gpu_prof.sh rn_fused --skip-gpt 1 --resnet-steps 8 > gpurun_out/prof_rn_fused.log 2>&1; echo "prof fused rc=$?"
FLAGS_conv_bn_fusion=0 bash tools/gpu_prof.sh rn_unfused --skip-gpt 1 --resnet-steps 8 > gpurun_out/prof_rn_unfused.log 2>&1; echo "prof unfused rc=$?"
for t in rn_fused rn_unfused; do
  f=$(find gpurun_out/prof_$t -name "*kernel_trace.csv" | head -1)
  python tools/prof_window.py --ms 150 --top 40 "$f" > gpurun_out/${t}_window.md 2>&1
  grep "img/s" gpurun_out/prof_$t/bench.log | tail -2; head -12 gpurun_out/${t}_window.md
done
