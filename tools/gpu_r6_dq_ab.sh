#!/bin/bash
# round-6: dQ kernel ring depth A/B (4 vs 5 slots) + the dS-route numerics test with 5 slots
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/dq_ab
for n in 4 5 4 5; do
  PA_FA_DQ_SLOTS=$n timeout -k 10 120 python -u tools/fa_bwd_time.py >> gpurun_out/dq_ab/ab.log 2>&1 || exit 1
done
cat gpurun_out/dq_ab/ab.log | grep PA_FA
PA_FA_DQ_SLOTS=5 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_attn.py -m gpu > gpurun_out/dq_ab/test.log 2>&1; rc=$?; tail -3 gpurun_out/dq_ab/test.log; exit $rc
