"""Join the per-process stage traces written with DX_STAGE_TRACE=<prefix>
(utils/tracing.py `stage`) on the request id and print, for each pair of
consecutive stages, the p50 / p90 / p99 gap in ms -- where the time between
the HTTP request arriving and its first token leaving goes.

    DX_STAGE_TRACE=/tmp/st python tools/frontend_scale.py ...
    python tools/stage_report.py /tmp/st
"""
from __future__ import annotations

import glob
import json
import sys
from collections import defaultdict

ORDER = ["http.recv", "cli.send:", "srv.recv:", "eng.arrival", "eng.admit", "eng.first", "srv.first:", "cli.first:",
         "http.first"]


def _rank(name: str) -> int:
    for i, p in enumerate(ORDER):
        if name.startswith(p):
            return i
    return len(ORDER)


def load(prefix: str) -> dict:
    reqs: dict = defaultdict(list)
    for path in glob.glob(f"{prefix}.*.jsonl"):
        with open(path) as f:
            for line in f:
                name, rid, t = json.loads(line)
                reqs[rid].append((t, name))
    return reqs


def report(prefix: str, t_from: float = 0.0) -> dict:
    reqs = load(prefix)
    gaps: dict = defaultdict(list)
    for rid, ev in reqs.items():
        ev.sort()
        if not ev or ev[0][0] < t_from or ev[0][1] != "http.recv" or ev[-1][1] != "http.first":
            continue
        for (t0, a), (t1, b) in zip(ev, ev[1:]):
            gaps[f"{a} -> {b}"].append((t1 - t0) * 1e3)
        gaps["TOTAL http.recv -> http.first"].append((ev[-1][0] - ev[0][0]) * 1e3)
    out = {}
    for k, v in sorted(gaps.items(), key=lambda kv: -sorted(kv[1])[len(kv[1]) // 2]):
        v.sort()
        out[k] = {"n": len(v), "p50": round(v[len(v) // 2], 2), "p90": round(v[int(len(v) * .9)], 2),
                  "p99": round(v[int(len(v) * .99)], 2)}
    return out


if __name__ == "__main__":
    r = report(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
    for k, v in r.items():
        print(f"{k:60s} n={v['n']:6d} p50={v['p50']:9.2f} p90={v['p90']:9.2f} p99={v['p99']:9.2f}")
