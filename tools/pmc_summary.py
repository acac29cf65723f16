"""Per-kernel PMC counter means from a rocprofv3 --pmc database (pmc_events view): one row per kernel name,
counter values summed over a dispatch's instances then averaged over dispatches; with GRBM_GUI_ACTIVE the
effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration).
    python tools/pmc_summary.py <db> [name filter]"""
import collections
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = db.execute("select dispatch_id, name, duration, counter_name, sum(counter_value) from pmc_events "
                      "group by dispatch_id, counter_name").fetchall()
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for did, name, d, cn, v in rows:
        if filt not in name:
            continue
        per[name][cn].append(v)
        dur[name][did] = d
    for name, cs in per.items():
        ds = list(dur[name].values())
        md = sum(ds) / len(ds)
        print(f"{name[:90]}  dispatches {len(ds)}  mean {md / 1e3:.1f} us")
        for cn in sorted(cs):
            m = sum(cs[cn]) / len(cs[cn])
            extra = ""
            if cn == "GRBM_GUI_ACTIVE" and md > 0:
                extra = f"   (clock {m / 8 / md:.2f} GHz)"
            print(f"    {cn:28s} {m:16.0f}{extra}")


if __name__ == "__main__":
    main()
