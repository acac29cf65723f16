#!/bin/bash
# Round 4 box 2: new GPU tests (layout autotune, side-stream native backward), ResNet-50 NHWC vs NCHW +
# layout autotune, LLaMA-2 7B static auto-parallel engine vs fleet dygraph kernel profiles.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=6
step pytest_new 600 python -u -m pytest tests/test_layout_autotune.py tests/test_autograd_engine.py -m gpu -x -v --timeout 300 --timeout-method thread
TAIL=5 step rn_nhwc 600 python bench.py --skip-gpt 1 --resnet-steps 10 --steps 1 --warmup 3
TAIL=5 step rn_nchw_autotune 600 python bench.py --skip-gpt 1 --resnet-steps 10 --steps 1 --warmup 3 --resnet-layout nchw-autotune
bash tools/gpu_prof.sh llama7b_static --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 2 --warmup 1 --resnet 0 > gpurun_out/prof_llama_static.log 2>&1; echo "prof static rc=$?"
python tools/prof_summary.py gpurun_out/prof_llama7b_static --top 30 > gpurun_out/llama7b_static_summary.md 2>&1
bash tools/gpu_prof.sh llama7b_fleet --model llama2-7b --llama-engine fleet --micro-batch 2 --accum 4 --seq-len 4096 --steps 2 --warmup 1 --resnet 0 > gpurun_out/prof_llama_fleet.log 2>&1; echo "prof fleet rc=$?"
python tools/prof_summary.py gpurun_out/prof_llama7b_fleet --top 30 > gpurun_out/llama7b_fleet_summary.md 2>&1
head -20 gpurun_out/llama7b_static_summary.md; head -20 gpurun_out/llama7b_fleet_summary.md
