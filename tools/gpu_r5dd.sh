#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=1 step rn_eager 400 python bench.py --skip-gpt 1 --resnet-steps 20 && \
TAIL=1 step rn_graph 400 python bench.py --skip-gpt 1 --resnet-steps 20 --resnet-graph 1 && \
TAIL=1 step rn_eager2 400 python bench.py --skip-gpt 1 --resnet-steps 20 && \
TAIL=1 step rn_graph2 400 python bench.py --skip-gpt 1 --resnet-steps 20 --resnet-graph 1
grep -h "img/s=" gpurun_out/rn_*.log
