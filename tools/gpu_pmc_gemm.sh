#!/bin/bash
# PMC passes (one counter set per run): ping-pong kernel vs hipBLASLt on the fc2-dgrad (both K-major) shape
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc_gemm"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU"
i=0
for C in "$C1" "$C2"; do
  i=$((i+1))
  for v in 0 1; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_gemm/v${v}_p$i" -o run -- \
      python3 "$R/tools/gemm_one.py" $v dgrad 4096 20480 5120 10 > "$R/gpurun_out/pmc_gemm/v${v}_p$i.log" 2>&1 || { echo "pmc v$v p$i failed"; tail -5 "$R/gpurun_out/pmc_gemm/v${v}_p$i.log"; exit 1; }
    echo "v$v p$i ok"
  done
done
