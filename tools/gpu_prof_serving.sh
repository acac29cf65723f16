#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/prof_serving"
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_serving" -o run -- \
  python3 "$R/tools/bench_serving.py" llama2-7b 32 512 64 > "$R/gpurun_out/prof_serving/bench.log" 2>&1
echo rc=$?
tail -3 "$R/gpurun_out/prof_serving/bench.log"
rm -f "$R"/gpurun_out/prof_serving/*kernel_trace.csv
ls -la "$R/gpurun_out/prof_serving"
