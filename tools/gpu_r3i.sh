#!/bin/bash
# round 3: MI355X op cost table for paddle.cost_model, gemm-epilogue pass latency, new CPU-tested modules on GPU
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4 step op_cost_table 600 python -u tools/gen_op_cost_table.py
TAIL=3 step pass_fusion 300 python -u tools/bench_pass_fusion.py
TAIL=4 step new_tests 300 python -u -m pytest tests/test_cost_model.py tests/test_dist_passes.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
