#!/bin/bash
# LayerNorm forward kernel form in the 13B step: rocprofv3 stats, rows kernel vs workgroup-per-row kernel
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
for v in 0 2; do
  PA_NORM_BWD_VARIANT=2 PA_NORM_FWD_VARIANT=$v bash tools/gpu_prof.sh normf_v$v --steps 1 --warmup 1 --resnet 0 > gpurun_out/prof_normf_v$v.log 2>&1 || exit 1
done
