#!/bin/bash
# round 3: new GPU tests, interpreter latency on GPU, whole suite, native-autograd-engine A/B on the 13B step
source "$(dirname "$0")/gpu_steps.sh"
TAIL=8 step new_tests 300 python -u -m pytest tests/test_bn_fused.py tests/test_pir_json.py tests/test_train_step_graph.py -m "gpu or not gpu" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAIL=3 step bench_interp 200 python -u tools/bench_interp.py
TAIL=6 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
export FLAGS_eager_backward_engine=native
TAIL=3 step bench_13b_native_engine 700 python bench.py --resnet 0 --steps 3 --warmup 1
