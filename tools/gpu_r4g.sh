#!/bin/bash
# Round 4 box 7: conv -> BN fusion parity + static hipGraph executor tests, ResNet-50 kernel windows with the
# fusion on and off, then the GPT-3 13B kernel profile.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6 step pytest_convbn 300 python -u -m pytest tests/test_conv_bn_fusion_gpu.py tests/test_production_geometry_gpu.py tests/test_static_graph_capture.py -m gpu -x -q --timeout 120 --timeout-method thread
bash tools/gpu_prof.sh rn_fused --skip-gpt 1 --resnet-steps 8 > gpurun_out/prof_rn_fused.log 2>&1; echo "prof fused rc=$?"
FLAGS_conv_bn_fusion=0 bash tools/gpu_prof.sh rn_unfused --skip-gpt 1 --resnet-steps 8 > gpurun_out/prof_rn_unfused.log 2>&1; echo "prof unfused rc=$?"
for t in rn_fused rn_unfused; do
  f=$(find gpurun_out/prof_$t -name "*kernel_trace.csv" | head -1)
  python tools/prof_window.py --ms 150 --top 40 "$f" > gpurun_out/${t}_window.md 2>&1
  grep "img/s\|backend per shape" gpurun_out/prof_$t/bench.log | tail -4; head -12 gpurun_out/${t}_window.md
done
bash tools/gpu_prof.sh gpt13b_r4 --steps 2 --warmup 1 --resnet 0 > gpurun_out/prof_gpt13b_r4.log 2>&1; echo "prof 13b rc=$?"
python tools/prof_summary.py gpurun_out/prof_gpt13b_r4 --top 60 > gpurun_out/gpt13b_r4_summary.md 2>&1; head -40 gpurun_out/gpt13b_r4_summary.md
