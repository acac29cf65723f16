#!/bin/bash
# end of round 5: 13B kernel stats (CSV) + default bench
source "$(dirname "$0")/gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$R"
TAIL=2 step prof13b_final 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof13b_final -o run -- python bench.py --resnet 0 --steps 3 --warmup 2 && \
find gpurun_out/prof13b_final -name "*kernel_trace.csv" -delete && \
TAIL=3 step bench_final 900 python bench.py
