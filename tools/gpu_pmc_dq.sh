#!/bin/bash
# round-6: PMC of the flash-attention dS-route backward kernels (B4 S2048 H40 causal), one pass per counter set
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc_dq"
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
C1="FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES"
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES"
C3="TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
i=0
for C in "$C1" "$C2" "$C3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$R/gpurun_out/pmc_dq/p$i" -o run -- \
    python3 "$R/tools/fa_dq_one.py" > "$R/gpurun_out/pmc_dq/p$i.log" 2>&1 || { echo "pmc p$i failed"; tail -5 "$R/gpurun_out/pmc_dq/p$i.log"; exit 1; }
  echo "p$i ok"
done
