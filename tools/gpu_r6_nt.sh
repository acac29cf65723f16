#!/bin/bash
# round-6: native-executor GPU tests (comm stream) + the default 13B bench on the committed tuning table
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
step nt_gpu2 300 python -u -m pytest tests/test_native_train_executor.py tests/test_fusion_passes.py tests/test_dwconv.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
step b13_table 400 python bench.py --resnet 0 --steps 3 --warmup 2
