#!/bin/bash
# PMC of the fc2 dgrad (TN) on the ping-pong, 4-wave K64 and hipBLASLt kernels
source "$(dirname "$0")/gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$R"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"
TAIL=3 step pmc1 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc $P1 -d gpurun_out/pmc1 -o run -- python3 tools/gemm_pmc_one.py
TAIL=3 step pmc2 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc $P2 -d gpurun_out/pmc2 -o run -- python3 tools/gemm_pmc_one.py
find gpurun_out/pmc1 gpurun_out/pmc2 -name "*.csv" | head
