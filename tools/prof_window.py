"""Steady-state kernel breakdown from a rocprofv3 kernel trace: only the kernels of the last ``--ms``
milliseconds of GPU time (skips autotuning / warm-up), grouped by category."""
import argparse
import csv


def cat(n):
    if "Cijk" in n:
        return "GEMM hipBLASLt"
    if "igemm" in n or "ck::" in n or "naive_conv" in n or "MIOpen" in n or "_ZN2ck" in n:
        return "conv MIOpen/CK"
    if "conv" in n.lower() or "gemm" in n.lower():
        return "GEMM/conv hand-written"
    if "bn_" in n:
        return "batch-norm hand-written"
    if "fa_" in n:
        return "attention hand-written"
    if "at::native" in n:
        return "ATen elementwise"
    return "other hand-written"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--ms", type=float, required=True)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    end = max(int(r["End_Timestamp"]) for r in rows)
    lo = end - a.ms * 1e6
    sel = [r for r in rows if int(r["Start_Timestamp"]) >= lo]
    tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel)
    by_cat, by_name = {}, {}
    for r in sel:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        by_cat[cat(r["Kernel_Name"])] = by_cat.get(cat(r["Kernel_Name"]), 0) + d
        k = r["Kernel_Name"][:120]
        c, t = by_name.get(k, (0, 0))
        by_name[k] = (c + 1, t + d)
    print(f"window {a.ms:.0f} ms, {len(sel)} kernels, busy {tot / 1e6:.1f} ms")
    for c, t in sorted(by_cat.items(), key=lambda x: -x[1]):
        print(f"  {c:26s} {t / 1e6:8.2f} ms {100 * t / tot:5.1f}%")
    for k, (c, t) in sorted(by_name.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"  {t / 1e6:8.2f} ms {c:5d}  {k}")


if __name__ == "__main__":
    main()
