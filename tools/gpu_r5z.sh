#!/bin/bash
# round 5: static engine on GPU with recompute (checkpointed segments + main grads) and selective recompute
source "$(dirname "$0")/gpu_steps.sh"
B="python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 1 --resnet 0"
TAIL=1 step static_rc 400 $B --recompute 1
grep -h "llama-static\]" gpurun_out/static_rc.log
