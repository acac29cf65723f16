#!/bin/bash
# gemm256 epilogue: one-pass bf16 staging (default) vs two fp32 halves (PA_GEMM_EPI_F32=1); tests then K sweeps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm.py > gpurun_out/pytest_gemm_epi.log 2>&1 || exit 1
for v in 0 1 0; do
  PA_GEMM_EPI_F32=$v timeout -k 10 300 python -u tools/bench_gemm_k_sweep.py 0,2,3 > gpurun_out/ksweep_epi$v.log 2>&1 || exit 1
  cp gpurun_out/ksweep_epi$v.log gpurun_out/ksweep_epi${v}_$(date +%s).log
done
