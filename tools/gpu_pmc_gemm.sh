#!/bin/bash
# PMC passes (one counter set per run) over the GEMM variants on the fc1 shape.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc_gemm"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
for v in 0 160 256; do
  timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv -d "$R/gpurun_out/pmc_gemm/v$v" -o run -- \
    python3 "$R/tools/gemm_one.py" $v fwd > "$R/gpurun_out/pmc_gemm/v$v.log" 2>&1 || { echo "pmc v$v failed rc=$?"; tail -5 "$R/gpurun_out/pmc_gemm/v$v.log"; exit 1; }
  echo "v$v ok"
done
