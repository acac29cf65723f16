"""Per-kernel time summary of a rocprofv3 --kernel-trace run stored as a rocpd sqlite database (``-o run`` ->
run_results.db): total / mean time and share of kernel time, grouped by kernel name (template arguments cut).

    python tools/prof_db_stats.py gpurun_out/prof13b/run_results.db [top]
"""
import collections
import re
import sqlite3
import sys


def stats(path):
    con = sqlite3.connect(path)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    rows = con.execute("select * from kernels").fetchall()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        d = dict(zip(cols, r))
        name = d.get("kernel_name") or d.get("name") or "?"
        name = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
        a = agg[name]
        a[0] += 1
        a[1] += (d["end"] - d["start"]) / 1e3
    return agg


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    agg = stats(path)
    total = sum(v[1] for v in agg.values())
    print(f"total kernel time {total / 1e3:.1f} ms over {sum(v[0] for v in agg.values())} dispatches")
    print(f"{'kernel':90s} {'calls':>7s} {'total ms':>10s} {'mean us':>9s} {'share':>6s}")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{k[:90]:90s} {n:7d} {t / 1e3:10.2f} {t / n:9.1f} {100 * t / total:5.1f}%")


if __name__ == "__main__":
    main()
