#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run. Usage: gpu_prof.sh <tag> <bench args...>
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
mkdir -p "$R/gpurun_out/prof_$TAG"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" "$@" > "$R/gpurun_out/prof_$TAG/bench.log" 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 "$R/gpurun_out/prof_$TAG/bench.log"
f=$(find "$R/gpurun_out/prof_$TAG" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -30 "$f" | cut -c1-250
exit $rc
