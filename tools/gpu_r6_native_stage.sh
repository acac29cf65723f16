#!/bin/bash
# round-6: static engine stages on the native executor — GPU tests, LLaMA-2 7B native vs Python replay, 70B proxy
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step ns_gpu 300 python -u -m pytest tests/test_static_engine_gpu.py tests/test_native_train_executor.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
step l7_native 500 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 2 --resnet 0
FLAGS_static_engine_native=0 step l7_python 500 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 2 --resnet 0
step l7_native_b 500 python bench.py --model llama2-7b --micro-batch 2 --accum 4 --seq-len 4096 --steps 3 --warmup 2 --resnet 0
step l70_native 600 python bench.py --model llama2-70b-stage --seq-len 4096 --micro-batch 1 --accum 8 --steps 2 --warmup 1 --resnet 0
