#!/bin/bash
# PMC counters for the flash-attention backward kernel (kernel-trace only; no sys/runtime trace).
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc_fa"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc_fa/counters.txt" 2>&1
rc=0
i=0
for set in "SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$R/gpurun_out/pmc_fa/set$i" -o run -- \
    python3 "$R/tools/abl_fa.py" > "$R/gpurun_out/pmc_fa/set$i.log" 2>&1
  rc=$?
  echo "set$i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
