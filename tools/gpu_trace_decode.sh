#!/bin/bash
# kernel trace of a short graph-decode run (order of kernels in one decode step)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/trace_decode"
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_decode" -o run -- \
  python3 "$R/tools/bench_serving.py" llama2-7b 32 512 8 > "$R/gpurun_out/trace_decode/bench.log" 2>&1
echo rc=$?
f=$(find "$R/gpurun_out/trace_decode" -name "*kernel_trace.csv" | head -1)
python3 - "$f" > "$R/gpurun_out/trace_decode/last_steps.txt" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-1400:]:
    print(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"][:110])
PY
rm -f "$f"
tail -2 "$R/gpurun_out/trace_decode/bench.log"
