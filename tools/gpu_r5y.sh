#!/bin/bash
# round 5: native executor data-parallel gradient hook + PIR control flow on GPU
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step nt_gpu 300 python -u -m pytest tests/test_native_train_executor.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider
