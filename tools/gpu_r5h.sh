#!/bin/bash
# native training executor + new ops on the GPU, then the static-program suites that now default to it
source "$(dirname "$0")/gpu_steps.sh"
TAIL=12 step native_exec 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_native_train_executor.py tests/test_qkv_rope_attention.py tests/test_reduced_attn_scores.py -m gpu
TAIL=8 step static_suites 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_static_graph_capture.py tests/test_static_jit.py tests/test_static_quantization.py tests/test_dist_passes.py tests/test_incubate.py tests/test_hip_kernels.py -m gpu
