#!/bin/bash
# same-box A/B of the GPT-3 13B step: the tree at the start of this session (ab_old/) vs the current tree
source "$(dirname "$0")/gpu_steps.sh"
TAIL=3
step bench_cur1 600 python bench.py --resnet 0
(cd ab_old && timeout -k 10 600 python bench.py --resnet 0 > ../gpurun_out/bench_old.log 2>&1); echo "== bench_old rc=$?"; grep "loss=" gpurun_out/bench_old.log
step bench_cur2 600 python bench.py --resnet 0
