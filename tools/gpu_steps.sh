#!/bin/bash
# Shared helper: run named GPU steps with per-step timeouts; stop at the first crash/timeout.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -${TAIL:-6}
  case $rc in 124|134|137|139) echo "FATAL in $name, stopping"; exit $rc;; esac
  return 0
}
