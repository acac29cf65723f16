#!/bin/bash
# round 3: C++ backward executor (_C_autograd) on the GPU: whole GPU suite under it, 13B + ResNet A/B
source "$(dirname "$0")/gpu_steps.sh"
export FLAGS_eager_backward_engine=native
TAIL=6 step pytest_gpu_native 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=3 step bench_13b_native_exec 700 python bench.py --resnet 0 --steps 3 --warmup 1
TAIL=4 step resnet_native_exec 600 python -u bench.py --skip-gpt 1 --resnet-steps 20
unset FLAGS_eager_backward_engine
TAIL=3 step bench_13b_torch_engine 700 python bench.py --resnet 0 --steps 3 --warmup 1
TAIL=4 step resnet_torch_engine 600 python -u bench.py --skip-gpt 1 --resnet-steps 20
