#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc_fa"
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"
i=0
for C in "$C1" "$C2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_fa/p$i" -o run -- \
    python3 "$R/tools/fa_one.py" > "$R/gpurun_out/pmc_fa/p$i.log" 2>&1 || { echo "pmc p$i failed"; tail -5 "$R/gpurun_out/pmc_fa/p$i.log"; exit 1; }
  echo "p$i ok"
done
