#!/bin/bash
# headline bench as the driver runs it, pairing microbench, weight-only dispatch bench, 13B rocprof summary
source "$(dirname "$0")/gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$R"
TAIL=3 step bench_default 600 python bench.py
TAIL=3 step bench_nopair 400 python bench.py --pair-wgrad 0 --resnet 0
TAIL=8 step wgrad_pair 200 python tools/bench_wgrad_epi.py pair
TAIL=30 step wo_bench 300 python tools/bench_wo.py
TAIL=3 step prof13b 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof13b -o run -- python bench.py --resnet 0 --steps 3 --warmup 2
