#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step test_graph_step 300 python -u -m pytest tests/test_train_step_graph.py -x -q --timeout 200 --timeout-method thread
TAIL=6 step resnet_graph 600 python bench.py --skip-gpt 1 --resnet-steps 20
