#!/bin/bash
# A/B: bias / norm-parameter gradients through autograd vs accumulated in the finalize kernels
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
PADDLE_AMD_VECTOR_MAIN_GRAD=0 step bench_vmg0 600 python bench.py --resnet 0
PADDLE_AMD_VECTOR_MAIN_GRAD=1 step bench_vmg1 600 python bench.py --resnet 0
PADDLE_AMD_VECTOR_MAIN_GRAD=0 step bench_vmg0b 600 python bench.py --resnet 0
