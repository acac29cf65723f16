#!/bin/bash
# round-6: ATen op census + kernel stats of a 2-layer GPT-3 13B-shaped step (mb 4 x accum 4) on the sharding-3 engine
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/census"
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/op_census.py --layers 2 > gpurun_out/census/census.log 2>&1 || { tail -20 gpurun_out/census/census.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/census/prof" -o run -- \
  python3 "$R/tools/op_census.py" --layers 2 > "$R/gpurun_out/census/prof.log" 2>&1 || { tail -20 "$R/gpurun_out/census/prof.log"; exit 1; }
echo done
