"""One bench.py GPT step under torch.profiler with Python stacks: which framework call sites launch the ATen
(non hand-written) kernels. Usage: python tools/profile_small_ops.py [bench args]. Outside bench's timed region."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["bench.py", "--steps", "1", "--warmup", "1", "--resnet", "0"] + sys.argv[1:]
import bench  # noqa: E402

_orig = bench.timed


def _prof_timed(step_fn, steps, warmup, dist_on):
    for _ in range(max(warmup, 1)):
        step_fn()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as p:
        step_fn()
        torch.cuda.synchronize()
    ka = p.key_averages(group_by_stack_n=8)
    rows = [e for e in ka if e.key.startswith("aten::") and e.self_device_time_total > 0]
    rows.sort(key=lambda e: -e.self_device_time_total)
    print("# ATen ops by self device time (one step), with their framework call sites", flush=True)
    for e in rows[:40]:
        stack = [s for s in (e.stack or []) if "paddlepaddle_amd" in s or "bench.py" in s][:4]
        print(f"{e.self_device_time_total / 1000:9.2f} ms  x{e.count:5d}  {e.key}")
        for s in stack:
            print(f"              {s}")
    sys.stdout.flush()
    return _orig(step_fn, steps, 0, dist_on)


bench.timed = _prof_timed
bench.main()
