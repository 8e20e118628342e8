"""Per-engine-step GPU time breakdown from a rocprofv3 kernel trace (rocpd
sqlite or kernel_trace.csv), for the timed window of a bench run.

  python tools/step_breakdown.py trace.db [last_seconds]

Splits the trace at every `embedding_kernel` dispatch (one per forward),
classifies each step as `decode` (no prefill attention) or `mixed`, and
prints per class: step count, mean wall span (embedding to next embedding),
mean GPU-busy time, and mean kernel time per kernel family.
"""
import re
import sqlite3
import sys
from collections import defaultdict

FAMILIES = [
    ("fused_mlp", r"gemm256_kernel"),
    ("hipblaslt", r"^Cijk_|^Custom_Cijk"),
    ("small_m_gemm", r"skinny_|dstream|splitk_reduce"),
    ("attn_decode", r"decode_attn|decode_reduce"),
    ("attn_prefill", r"prefill_attn"),
    ("rmsnorm", r"rmsnorm|row_rrms"),
    ("rope_cache", r"rope_cache"),
    ("silu_mul", r"silu_and_mul"),
    ("sampling", r"sample_|penalt"),
    ("embedding", r"embedding_kernel"),
    ("allreduce", r"custom_ar|nccl|rccl"),
]


def family(name: str) -> str:
    for f, pat in FAMILIES:
        if re.search(pat, name):
            return f
    return "other"


def load(path):
    if path.endswith(".csv"):
        import csv
        with open(path) as f:
            rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(f)]
        return sorted(rows, key=lambda r: r[1])
    db = sqlite3.connect(path)
    q = ("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    try:
        return db.execute(q).fetchall()
    except sqlite3.OperationalError:
        return db.execute(q.replace("s.display_name", "s.kernel_name")).fetchall()


def breakdown(rows, last_s=None):
    if last_s:
        t_end = max(e for _, _, e in rows)
        rows = [r for r in rows if r[1] >= t_end - last_s * 1e9]
    starts = [i for i, (n, _, _) in enumerate(rows) if "embedding_kernel" in n]
    steps = []
    for a, b in zip(starts, starts[1:]):
        ks = rows[a:b]
        wall = rows[b][1] - rows[a][1]
        busy, cur_s, cur_e = 0, None, None
        fam = defaultdict(float)
        for n, s, e in ks:
            fam[family(n)] += e - s
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        kind = "mixed" if fam.get("attn_prefill") else "decode"
        steps.append((kind, wall, busy, fam))
    out = {}
    for kind in ("decode", "mixed"):
        sel = [s for s in steps if s[0] == kind]
        if not sel:
            continue
        n = len(sel)
        fam = defaultdict(float)
        for _, _, _, f in sel:
            for k, v in f.items():
                fam[k] += v
        out[kind] = {"steps": n, "wall_ms": sum(s[1] for s in sel) / n / 1e6,
                     "busy_ms": sum(s[2] for s in sel) / n / 1e6,
                     "families_ms": {k: round(v / n / 1e6, 3) for k, v in sorted(fam.items(), key=lambda kv: -kv[1])}}
    return out


def report(out) -> str:
    lines = []
    for kind, d in out.items():
        lines.append(f"{kind}: {d['steps']} steps, wall {d['wall_ms']:.2f} ms/step, GPU busy {d['busy_ms']:.2f} ms/step "
                     f"({100 * d['busy_ms'] / d['wall_ms']:.1f} %)")
        for k, v in d["families_ms"].items():
            lines.append(f"    {k:14s} {v:8.3f} ms  {100 * v / d['wall_ms']:5.1f} %")
    return "\n".join(lines)


if __name__ == "__main__":
    rows = load(sys.argv[1])
    print(report(breakdown(rows, float(sys.argv[2]) if len(sys.argv) > 2 else None)))
