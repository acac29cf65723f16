#!/bin/bash
# GEMM solution tuning experiment: run the 13B bench once with PyTorch TunableOp tuning every
# hipBLASLt/rocBLAS solution per GEMM shape (results -> gpurun_out/tunableop.csv), then re-run
# with tuning off using that file, plus the static/jit GPU tests.
source "$(dirname "$0")/gpu_steps.sh"
step pytest_static_gpu 600 python -m pytest tests/test_static_jit.py tests/test_llama.py -m gpu -x -q
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_FILENAME="$R/gpurun_out/tunableop.csv"
export PYTORCH_TUNABLEOP_TUNING=1
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20
export PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5
step bench_tune 1000 python bench.py --resnet 0 --steps 2 --warmup 2
export PYTORCH_TUNABLEOP_TUNING=0
step bench_tuned 600 python bench.py --resnet 0 --steps 3 --warmup 1
ls -la gpurun_out/tunableop*.csv
