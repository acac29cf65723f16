#!/bin/bash
# same-box A/B of the LayerNorm kernel form in the GPT-3 13B step: wide (default) vs rows, twice each
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/norm_ab.log
for v in 0 1 0 1; do
  PA_NORM_ROWS_ONLY=$v timeout -k 10 400 python bench.py --resnet 0 --steps 3 --warmup 2 > gpurun_out/norm_ab_$v.log 2>&1 || exit 1
  echo "rows_only=$v $(grep '"value"' gpurun_out/norm_ab_$v.log | cut -c80-140)" >> gpurun_out/norm_ab.log
done
