#!/bin/bash
# round-6: LLaMA-2 7B static engine with recompute, native stages vs Python replay (same box)
source "$(dirname "$0")/gpu_steps.sh"
TAIL=2
step l7rc_native 500 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 2 --resnet 0 --recompute 1
FLAGS_static_engine_native=0 step l7rc_python 500 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 2 --resnet 0 --recompute 1
