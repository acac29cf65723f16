#!/bin/bash
# LLaMA-7B A/B on one box: fleet with / without the fused qkv-RoPE-attention op; static engine with each program pass
source "$(dirname "$0")/gpu_steps.sh"
B="python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0"
TAIL=2 step fleet_fused 300 $B --llama-engine fleet --llama-fused-attn 1
TAIL=2 step fleet_unfused 300 $B --llama-engine fleet --llama-fused-attn 0
TAIL=2 step static_none 300 $B --static-passes none
TAIL=2 step static_rms 300 $B --static-passes rms_norm_residual
TAIL=2 step static_sib 300 $B --static-passes sibling_linears
TAIL=2 step fleet_fused2 300 $B --llama-engine fleet --llama-fused-attn 1
TAIL=12 step native_exec 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_native_train_executor.py -m gpu
