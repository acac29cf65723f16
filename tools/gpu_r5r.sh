#!/bin/bash
# round 5: wgrad layout A/B + the new native-interpreter control-flow GPU test
source "$(dirname "$0")/gpu_steps.sh"
TAIL=20 step wgrad_layout 300 python -u tools/bench_wgrad_layout.py 20 && \
TAIL=15 step cf_gpu 300 python -u -m pytest tests/test_pir_json.py tests/test_native_interp_kernels.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider
