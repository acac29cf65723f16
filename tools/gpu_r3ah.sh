#!/bin/bash
# ResNet-50 steady-state kernel trace after the skinny conv family; hipGraph-replayed ResNet step sanity.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
bash tools/gpu_prof.sh resnet50_r3c --skip-gpt 1 --resnet-steps 8 > gpurun_out/prof_rn.log 2>&1; echo "prof rc=$?"
step resnet_graph 600 python bench.py --skip-gpt 1 --resnet-steps 10 --resnet-graph 1
