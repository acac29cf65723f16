#!/bin/bash
# Round 4: LLaMA-2 70B single-layer fwd+bwd throughput and its rocprofv3 kernel summary
source "$(dirname "$0")/gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAIL=2 step llama70b_layer 300 python tools/bench_llama70b_layer.py && \
TAIL=2 step llama70b_layer_s8k 300 python tools/bench_llama70b_layer.py --seq 8192 && \
TAIL=2 step llama70b_layer_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_l70 -o l70 -- python tools/bench_llama70b_layer.py --steps 5
