#!/bin/bash
# round 3: FA backward 16-keys-per-wave kernel (numerics under the existing FA tests + timing), depthwise conv
# kernels, whole GPU suite, smoke
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4 step fa16_tests 400 env PA_FA_BWD16=1 python -u -m pytest tests/test_flash_attn.py tests/test_flash_attn_ext.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=6 step fa16_bench 300 python -u tools/bench_fa_bwd16.py
TAIL=4 step dwconv_tests 300 python -u -m pytest tests/test_dwconv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=10 step dwconv_bench 300 python -u tools/bench_dwconv.py
TAIL=6 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=3 step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
