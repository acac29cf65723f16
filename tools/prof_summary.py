"""Summarize a rocprofv3 `--kernel-trace --stats` run into a small markdown table for profiles/.

Usage: python tools/prof_summary.py gpurun_out/prof_TAG [--top 25] > profiles/TAG.md
Kernels are grouped into categories (GEMM library, our HIP kernels, PyTorch elementwise, RCCL...) so
the share of time spent outside hand-written kernels is visible at a glance.
"""
import argparse
import csv
import glob
import os
import re

CATS = [
    ("bn/bn+relu(+add) (HIP)", re.compile(r"bn_(reduce|apply|bwd_apply|fwd_finalize|bwd_finalize)_k")),
    ("maxpool NHWC (HIP)", re.compile(r"maxpool_nhwc_(fwd|bwd)_k")),
    ("miopen/ck(conv/bn)", re.compile(r"miopen|igemm|naive_conv|batchnorm|grouped_conv|SubTensorOp|MIOpen", re.I)),
    ("GEMM hipBLASLt/rocBLAS (vendor)", re.compile(r"^Cijk_|^Custom_Cijk|rocblas|hipblaslt", re.I)),
    ("GEMM/conv hand-written (HIP)", re.compile(r"gemm256_kernel|gemm_bf16_kernel|gemm3s_kernel|gemm_tail_reduce|"
                                                r"grouped_gemm|gemm_smallm|conv_|implicit_gemm|gemm")),
    ("flash_attn(HIP)", re.compile(r"fa_(fwd|bwd)|fa_delta|dq_convert")),
    ("norm(HIP)", re.compile(r"norm_(fwd|bwd)|layer_?norm|rms_?norm")),
    ("softmax/CE(HIP)", re.compile(r"softmax|xent|\bce_|_ce_")),
    ("epilogue/act/dropout(HIP)", re.compile(r"gelu|swiglu|rope|colsum|dropout|bias_")),
    ("optimizer(HIP)", re.compile(r"adamw|sq_norm|momentum")),
    ("rccl", re.compile(r"nccl|rccl|ncclDevKernel", re.I)),
    ("torch elementwise/reduce", re.compile(r"at::native|elementwise|reduce_kernel|vectorized")),
]


def category(name):
    for c, rx in CATS:
        if rx.search(name):
            return c
    return "other"


def _window_rows(d, last_ms):
    """kernel_stats-shaped rows rebuilt from kernel_trace.csv, restricted to the trace's last ``last_ms``."""
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not f:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    tr = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f[0]))]
    t_end = max(e for _, _, e in tr)
    agg = {}
    for n, s, e in tr:
        if s >= t_end - last_ms * 1e6:
            c, t = agg.get(n, (0, 0))
            agg[n] = (c + 1, t + e - s)
    tot = sum(t for _, t in agg.values()) or 1
    return [{"Name": n, "Calls": c, "TotalDurationNs": t, "AverageNs": t / c, "Percentage": 100.0 * t / tot}
            for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--last-ms", type=float, default=0.0,
                    help="only kernels that start in the last N ms of the trace (steady-state steps, excluding "
                         "one-time per-shape tuning such as the MIOpen find runs)")
    a = ap.parse_args()
    if a.last_ms > 0:
        rows = _window_rows(a.dir, a.last_ms)
    else:
        f = sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True))
        if not f:
            raise SystemExit(f"no kernel_stats.csv under {a.dir}")
        rows = list(csv.DictReader(open(f[0])))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    cats = {}
    for r in rows:
        c = category(r["Name"])
        cats[c] = cats.get(c, 0.0) + float(r["TotalDurationNs"])
    print(f"# rocprofv3 kernel summary: `{os.path.basename(a.dir.rstrip('/'))}`\n")
    log = os.path.join(a.dir, "bench.log")
    if os.path.exists(log):
        js = [l for l in open(log) if l.startswith("{")]
        if js:
            print("bench line:\n\n```\n" + js[-1].strip() + "\n```\n")
    print(f"Total GPU kernel time: {total / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} launches\n")
    print("| category | ms | % |\n|---|---:|---:|")
    for c, v in sorted(cats.items(), key=lambda kv: -kv[1]):
        print(f"| {c} | {v / 1e6:.1f} | {100 * v / total:.1f} |")
    print(f"\n## Top {a.top} kernels\n")
    print("| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    for r in rows[:a.top]:
        n = r["Name"]
        n = n if len(n) <= 90 else n[:87] + "..."
        n = n.replace("|", "/")
        print(f"| `{n}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.1f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main()
