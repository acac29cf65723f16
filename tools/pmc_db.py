"""Summarise a rocprofv3 (rocpd sqlite) PMC run: per kernel (name prefix), mean duration and mean counter values."""
import collections
import sqlite3
import sys


def summarise(path, match=None):
    con = sqlite3.connect(path)
    cur = con.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(counters_collection)")]
    rows = cur.execute("select * from counters_collection").fetchall()
    name_i = cols.index("kernel_name") if "kernel_name" in cols else None
    cn_i, val_i, disp_i = cols.index("counter_name"), cols.index("value"), cols.index("dispatch_id")
    dur = {}
    for r in cur.execute("select id, start, end, name from kernels" if False else "select * from kernels"):
        pass
    kcols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    for r in cur.execute("select * from kernels"):
        d = dict(zip(kcols, r))
        dur[d.get("dispatch_id", d.get("id"))] = (d["end"] - d["start"], d.get("kernel_name") or d.get("name"))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        did = r[disp_i]
        kname = r[name_i] if name_i is not None else dur.get(did, (0, "?"))[1]
        agg[kname][r[cn_i]].append(r[val_i])
        agg[kname]["__disp"].append(did)
    out = {}
    for k, d in agg.items():
        if match and not any(m in k for m in match):
            continue
        disp = sorted(set(d.pop("__disp")))
        n = len(disp)
        durs = [dur[x][0] for x in disp if x in dur]
        out[k] = {c: sum(v) / n for c, v in d.items()}
        out[k]["dur_us"] = sum(durs) / len(durs) / 1e3 if durs else 0
        out[k]["n"] = n
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for k, d in summarise(p).items():
            print(k[:90])
            print("   " + ", ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
