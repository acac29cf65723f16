#!/bin/bash
# ResNet-50 steady-state kernel trace + PMC passes of the skinny 3x3 conv / 1x1 GEMM.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/pmcsk
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_prof.sh resnet50_r3b --skip-gpt 1 --resnet-steps 8 || exit 1
cd /tmp && export TMPDIR=/tmp
C1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"
C2="TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
i=0
for C in "$C1" "$C2"; do
  i=$((i+1))
  for v in conv gemm; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmcsk/${v}_p$i" -o run -- \
      python3 "$R/tools/conv_one.py" $v 10 > "$R/gpurun_out/pmcsk/${v}_p$i.log" 2>&1 || { echo "pmc $v p$i failed"; tail -5 "$R/gpurun_out/pmcsk/${v}_p$i.log"; exit 1; }
    echo "$v p$i ok"
  done
done
