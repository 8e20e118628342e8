"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) or CSV into a
per-kernel table: calls, total ms, mean us, % of GPU time."""
import csv
import sqlite3
import sys
from collections import defaultdict


def intervals_db(path):
    db = sqlite3.connect(path)
    return sorted(db.execute("select start, end from rocpd_kernel_dispatch").fetchall())


def busy_report(iv, last_s: float) -> str:
    """GPU busy fraction over the last `last_s` seconds of the trace (the
    timed window of a bench run) and the largest idle gaps."""
    t_end = max(e for _, e in iv)
    t0 = t_end - last_s * 1e9
    iv = [(max(s, t0), e) for s, e in iv if e > t0]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - iv[0][0]
    gaps.sort(reverse=True)
    big = [g for g in gaps if g > 50e3]
    return (f"window {span/1e9:.2f} s: GPU busy {busy/span*100:.1f} %, idle {(span-busy)/1e6:.1f} ms in {len(gaps)} gaps; "
            f"gaps > 50 us: {len(big)} totalling {sum(big)/1e6:.1f} ms; largest (us): "
            + ", ".join(f"{g/1e3:.0f}" for g in gaps[:8]))


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
    if len(sys.argv) > 2 and sys.argv[2] == "--busy":
        print(busy_report(intervals_db(p), float(sys.argv[3])))
        sys.exit(0)
    rows = from_db(p) if p.endswith(".db") else from_csv(p)
    print(summarize(rows, int(sys.argv[2]) if len(sys.argv) > 2 else 40))
