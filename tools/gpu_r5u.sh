#!/bin/bash
# round 5: kernel-level comparison LLaMA-2 7B static engine vs fleet (rocprofv3 kernel stats, CSV)
source "$(dirname "$0")/gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$R"
B="bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0"
TAIL=2 step prof_static 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l7s -o run -- python $B && \
TAIL=2 step prof_fleet 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l7f -o run -- python $B --llama-engine fleet
find gpurun_out/prof_l7s gpurun_out/prof_l7f -name "*kernel_trace.csv" -delete
ls -R gpurun_out/prof_l7s | head
