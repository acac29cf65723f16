#!/bin/bash
# ablations + PMC passes of the 4-wave GEMM vs the ping-pong kernel on the fwd shape 4096 x 20480 x 5120
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/pmc4w
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python tools/bench_gemm_abl.py > gpurun_out/gemm_abl.log 2>&1 || { echo "abl failed"; tail gpurun_out/gemm_abl.log; exit 1; }
cat gpurun_out/gemm_abl.log
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"
i=0
for C in "$C1" "$C2"; do
  i=$((i+1))
  for v in 1 2; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc4w/v${v}_p$i" -o run -- \
      python3 "$R/tools/gemm_one.py" $v fwd 4096 5120 20480 10 > "$R/gpurun_out/pmc4w/v${v}_p$i.log" 2>&1 || { echo "pmc v$v p$i failed"; tail -5 "$R/gpurun_out/pmc4w/v${v}_p$i.log"; exit 1; }
    echo "v$v p$i ok"
  done
done
