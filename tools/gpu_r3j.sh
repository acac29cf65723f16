#!/bin/bash
# round 3: op cost table into gpurun_out (copied into the package), norm without affine params, ResNet profile
source "$(dirname "$0")/gpu_steps.sh"
TAIL=2 step op_cost_table 600 python -u tools/gen_op_cost_table.py --out gpurun_out/mi355x_op_benchmark.json
TAIL=4 step norm_tests 300 python -u -m pytest tests/test_hip_kernels.py -k "norm" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=4 step resnet_bench 600 python -u bench.py --skip-gpt 1 --resnet-steps 20
TAIL=3 step resnet_prof 900 bash tools/gpu_prof.sh resnet50_r3 --skip-gpt 1 --resnet-steps 8
f=$(find gpurun_out/prof_resnet50_r3 -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python tools/prof_window.py "$f" --ms 150 --top 30 > gpurun_out/resnet50_r3_window.txt && cat gpurun_out/resnet50_r3_window.txt | head -40
rm -f gpurun_out/prof_resnet50_r3/*/*kernel_trace.csv 2>/dev/null; true
