#!/bin/bash
# ablations + L2 / wave PMC passes of hipBLASLt (0), ping-pong (1), 4-wave (2) on fwd 4096 x 20480 x 5120
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/pmc4w2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python tools/bench_gemm_abl.py > gpurun_out/gemm_abl2.log 2>&1 || { echo "abl failed"; tail gpurun_out/gemm_abl2.log; exit 1; }
cat gpurun_out/gemm_abl2.log
cd /tmp && export TMPDIR=/tmp
C1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"
C2="TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
i=0
for C in "$C1" "$C2"; do
  i=$((i+1))
  for v in 0 1 2; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc4w2/v${v}_p$i" -o run -- \
      python3 "$R/tools/gemm_one.py" $v fwd 4096 5120 20480 10 > "$R/gpurun_out/pmc4w2/v${v}_p$i.log" 2>&1 || { echo "pmc v$v p$i failed"; tail -5 "$R/gpurun_out/pmc4w2/v${v}_p$i.log"; exit 1; }
    echo "v$v p$i ok"
  done
done
