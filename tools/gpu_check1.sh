#!/bin/bash
# First GPU validation pass: kernel numerics, smoke, a short 1.3B bench. Stops at any crash/timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "FATAL in $name, stopping"; exit $rc;; esac
  return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step smoke 300 python __graft_entry__.py smoke
step bench_1p3b 600 python bench.py --model gpt3-1.3b --micro-batch 8 --steps 4 --warmup 2 --resnet 1 --resnet-steps 10
