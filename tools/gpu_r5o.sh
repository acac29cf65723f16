#!/bin/bash
# rocprof kernel stats (CSV summaries only; traces deleted to stay under the copy-back limit)
source "$(dirname "$0")/gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$R"
B="python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0"
TAIL=1 step l7_static 300 $B
TAIL=2 step prof_l70 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l70 -o run -- python tools/bench_llama70b_layer.py
TAIL=2 step prof13b 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof13b_fix -o run -- python bench.py --resnet 0 --steps 3 --warmup 2
TAIL=2 step prof_l7 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l7 -o run -- $B --llama-engine fleet
find gpurun_out -name "*kernel_trace.csv" -delete
ls -la gpurun_out/prof_l70 gpurun_out/prof13b_fix gpurun_out/prof_l7
