#!/bin/bash
# segmented GEMMs / multi_linear / pairing / guards tests, pairing microbench, LLaMA-7B static vs fleet (same box)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step r5_tests 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_segmented_gemm_gpu.py tests/test_wgrad_pairing_gpu.py tests/test_native_interp_kernels.py tests/test_static_graph_capture.py tests/test_llama.py tests/test_weight_only_quant.py tests/test_qkv_rope_attention.py tests/test_hip_kernels.py -m gpu
TAIL=6 step wgrad_pair 300 python tools/bench_wgrad_epi.py pair
TAIL=30 step wo_bench 400 python tools/bench_wo.py
TAIL=3 step llama7b_static 900 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0
TAIL=3 step llama7b_fleet 900 python bench.py --model llama2-7b --llama-engine fleet --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0
