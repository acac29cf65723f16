#!/bin/bash
# round-5 batch g: part 1 = new-op GPU tests + LLaMA-7B static vs fleet (same box); part 2 = the 70B PP4xTP2 stage
# proxy (with and without static-engine recompute) + microbenches
source "$(dirname "$0")/gpu_steps.sh"
if [ "${1:-1}" = 1 ]; then
TAIL=8 step r5_tests 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_native_train_executor.py tests/test_qkv_rope_attention.py tests/test_reduced_attn_scores.py tests/test_hip_kernels.py tests/test_segmented_gemm_gpu.py tests/test_wgrad_pairing_gpu.py tests/test_native_interp_kernels.py tests/test_static_graph_capture.py tests/test_llama.py tests/test_weight_only_quant.py -m gpu
TAIL=3 step llama7b_fleet 400 python bench.py --model llama2-7b --llama-engine fleet --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0
TAIL=3 step llama7b_static 400 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0
else
TAIL=3 step llama70b_stage 600 python bench.py --model llama2-70b-stage --micro-batch 1 --accum 4 --seq-len 4096 --steps 2 --warmup 1 --resnet 0
TAIL=3 step llama70b_stage_rc 600 python bench.py --model llama2-70b-stage --micro-batch 1 --accum 4 --seq-len 4096 --steps 2 --warmup 1 --resnet 0 --recompute 1
TAIL=6 step wgrad_pair 200 python tools/bench_wgrad_epi.py pair
TAIL=30 step wo_bench 300 python tools/bench_wo.py
fi
