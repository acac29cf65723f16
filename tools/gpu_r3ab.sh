#!/bin/bash
# FA backward default = 16-key kernel: FA test files, GPT-3 13B A/B (16-key default vs PA_FA_BWD16=0) on one box.
source "$(dirname "$0")/gpu_steps.sh"
TAIL=4
step pytest_fa 300 python -u -m pytest tests/test_flash_attn.py tests/test_flash_attn_ext.py tests/test_serving_ops.py -m gpu -q -x --timeout 120 --timeout-method thread
step gpt_k16 600 python bench.py --resnet 0 --steps 5 --warmup 2
PA_FA_BWD16=0 step gpt_4wave 600 python bench.py --resnet 0 --steps 5 --warmup 2
step gpt_k16_again 600 python bench.py --resnet 0 --steps 5 --warmup 2
