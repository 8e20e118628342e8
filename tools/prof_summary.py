"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) or CSV into a
per-kernel table: calls, total ms, mean us, % of GPU time."""
import csv
import sqlite3
import sys
from collections import defaultdict


def from_db(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(rocpd_kernel_dispatch)")]
    q = ("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    try:
        rows = cur.execute(q).fetchall()
    except sqlite3.OperationalError:
        q = q.replace("s.display_name", "s.kernel_name")
        rows = cur.execute(q).fetchall()
    return [(n, (e - s) / 1e3) for n, s, e in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return out


def summarize(rows, top=40, shorten=110):
    agg = defaultdict(lambda: [0, 0.0])
    for n, us in rows:
        a = agg[n]
        a[0] += 1
        a[1] += us
    total = sum(v[1] for v in agg.values())
    lines = [f"total GPU kernel time: {total/1e3:.2f} ms over {sum(v[0] for v in agg.values())} dispatches", "",
             f"{'%':>6} {'total_ms':>10} {'calls':>7} {'mean_us':>9}  kernel"]
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        lines.append(f"{100*t/total:6.2f} {t/1e3:10.2f} {c:7d} {t/c:9.1f}  {n[:shorten]}")
    return "\n".join(lines)


if __name__ == "__main__":
    p = sys.argv[1]
    rows = from_db(p) if p.endswith(".db") else from_csv(p)
    print(summarize(rows, int(sys.argv[2]) if len(sys.argv) > 2 else 40))
