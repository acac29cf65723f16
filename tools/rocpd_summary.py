"""Per-kernel summary (calls, total / mean time, share) from a rocprofv3 SQLite database (rocpd schema), for runs
made without --output-format csv. Usage: python tools/rocpd_summary.py run_results.db [top] [--grid]  (--grid: one row per kernel and grid size)"""
import sqlite3
import sys


def summary(path, top=40, by_grid=False):
    c = sqlite3.connect(path)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    key = "s.kernel_name || ' grid=' || d.grid_size_x" if by_grid else "s.kernel_name"
    rows = c.execute(f"select {key}, count(*), sum(d.end - d.start) from {disp} d join {sym} s "
                     f"on d.kernel_id = s.id group by {key} order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    print(f"{'share':>6} {'calls':>6} {'total ms':>10} {'mean us':>9}  kernel")
    for name, n, t in rows[:top]:
        print(f"{100 * t / tot:6.2f} {n:6d} {t / 1e6:10.3f} {t / n / 1e3:9.1f}  {name[:150]}")
    print(f"total kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches")


if __name__ == "__main__":
    summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40, "--grid" in sys.argv)
