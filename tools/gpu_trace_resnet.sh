#!/bin/bash
# kernel trace of the ResNet-50 bench; summarise only the last 300 ms (steady-state steps, after
# MIOpen's first-call solver search and the conv backend tuning of the warmup)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/trace_resnet"
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_resnet" -o run -- \
  python3 "$R/bench.py" --skip-gpt 1 --resnet-steps 20 > "$R/gpurun_out/trace_resnet/bench.log" 2>&1
echo rc=$?
f=$(find "$R/gpurun_out/trace_resnet" -name "*kernel_trace.csv" | head -1)
python3 - "$f" > "$R/gpurun_out/trace_resnet/steady.txt" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
end = max(int(r["End_Timestamp"]) for r in rows)
win = [r for r in rows if int(r["Start_Timestamp"]) >= end - 300_000_000]
t = collections.Counter(); c = collections.Counter()
for r in win:
    k = r["Kernel_Name"][:120]
    t[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"]); c[k] += 1
tot = sum(t.values())
print(f"window 300 ms: {len(win)} kernels, busy {tot/1e6:.1f} ms")
for k, v in t.most_common(40):
    print(f"{v/1e6:8.2f} ms {100*v/tot:5.1f}% {c[k]:5d}x {k}")
PY
rm -f "$f"
grep -v "^W\|^I\|^E" "$R/gpurun_out/trace_resnet/bench.log" | tail -3
