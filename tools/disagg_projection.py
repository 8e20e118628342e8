#!/usr/bin/env python3
"""Disaggregated vs aggregated throughput per GPU at matched tok/s/user, projected
from single-GPU measurements -- the reference's comparison
(docs/architecture.md:57-61: disagg 1.3x agg at ~50 tok/s/user; method
examples/llm/benchmarks/perf.sh:17-54: concurrency sweep, throughput/GPU vs
tok/s/user).

Inputs (all measured on one MI355X with the current kernels):
* the aggregated sweep: `bench.py --sweep ...` (one engine, C streams);
* decode-role sweeps: `bench.py --sweep ... --remote-frac q` -- the same engine
  with a fraction q of the prompts "remotely prefilled" (KV taken as landed),
  i.e. the decode GPU of an xPyD layout that prefills the other 1 - q itself
  (conditional disaggregation; q = 1: always remote);
* the prefill role: `tools/role_bench.py --role prefill` (prompts/s of a
  prefill-only engine at the ISL).

Model, per (prefill GPU, decode GPU) pair of an xPyD layout with x = y (the
BASELINE layouts 1P1D..4P4D; the shared prefill queue spreads remote prompts
over the x prefill GPUs, so the pair model holds for every k = x = y): a decode
point (q, C) with output M tok/s and u tok/s/user needs q * M / OSL remote
prompts/s; it is feasible when that is at most P (the prefill GPU's rate), and
gives M / 2 output tok/s per GPU at u.  When q = 1 demands more than P, the
decode GPU runs at the concurrency where q * M / OSL = P (interpolated along its
curve): prefill-bound.

The P->D transfer is charged, conservatively, as if it
were not overlapped with anything: every remote prompt costs the prefill GPU
its prefill time x (1 + pack overhead) + the wire time of its KV bytes over
ONE xGMI link (ISL x KV bytes per token / link GB/s; default 76.5 GB/s, half
of the 153 GB/s bidirectional link rate), and the decode GPU `unpack_ms`
(measured: prefill forwards at 1.007x their transfer-free time with the
layer-streamed packs, the unpack ~0.1 ms per ISL-3000 request:
profiles/r4_loopback_1p1d.json).  In the real pipeline the wire time rides
under the prefill forward (layer-streamed WRITE), so this understates xPyD.

Everything this tool prints is a PROJECTION from single-GPU role
measurements, not a measured multi-GPU result.  A target tok/s/user at which
the aggregated engine has no operating point gets no ratio.

Output: JSON with every projected point and, per target tok/s/user, the best
aggregated and disaggregated tok/s/GPU (frontier interpolation), plus a text
table.
"""
from __future__ import annotations

import argparse
import json


def _load_points(path: str) -> tuple[float, list[dict]]:
    d = json.load(open(path))
    if "points" not in d:  # a file of JSON lines: the last one with points
        raise SystemExit(f"{path}: no sweep points")
    return float(d.get("remote_frac", 0.0) or 0.0), d["points"]


def _interp(x0, y0, x1, y1, x):
    return y0 if x1 == x0 else y0 + (y1 - y0) * (x - x0) / (x1 - x0)


def frontier(points: list[tuple[float, float]], target: float) -> float | None:
    """Throughput at tok/s/user = target on the Pareto frontier of (u, tput)
    points (no other point is better in both), linear between the two
    frontier points around the target (intermediate concurrencies); None when
    no point reaches the target."""
    front = []
    for u, t in sorted(points, key=lambda p: (-p[0], -p[1])):  # by u descending: keep rising throughput
        if not front or t > front[-1][1]:
            front.append((u, t))
    front.sort()
    hi = [p for p in front if p[0] >= target]
    if not hi:
        return None
    u1, t1 = hi[0]
    lo = [p for p in front if p[0] < target]
    if not lo:
        return t1
    u0, t0 = lo[-1]
    return _interp(u0, t0, u1, t1, target)


def charged_rates(prompts_s: float, isl: int, kv_bytes_per_token: int, link_GBps: float, pack_overhead: float,
                  unpack_ms: float) -> dict:
    """The transfer term: the prefill GPU's effective prompts/s with each
    prompt's pack overhead and wire time charged serially, and the decode
    GPU's unpack seconds per remote prompt."""
    wire_s = isl * kv_bytes_per_token / (link_GBps * 1e9) if link_GBps else 0.0
    per_prompt = (1.0 / prompts_s) * (1.0 + pack_overhead) + wire_s
    return {"prefill_prompts_s_measured": prompts_s, "wire_ms": round(wire_s * 1e3, 3),
            "kv_mb_per_prompt": round(isl * kv_bytes_per_token / 1e6, 1), "pack_overhead": pack_overhead,
            "unpack_ms": unpack_ms, "prefill_prompts_s_charged": 1.0 / per_prompt}


def project(agg: list[dict], decode: dict[float, list[dict]], prompts_s: float, osl: int,
            unpack_ms: float = 0.0) -> dict:
    """`prompts_s`: the prefill GPU's rate with the transfer already charged
    (charged_rates); `unpack_ms`: decode-GPU time per remote prompt."""
    out = {"agg": [], "disagg": []}
    if unpack_ms:  # the decode GPU spends unpack_ms per remote prompt: its tok/s scale by 1 / (1 + demand x unpack)
        scaled = {}
        for q, pts in decode.items():
            scaled[q] = []
            for p in pts:
                if p.get("tok_s_user"):
                    f = 1.0 + q * p["tok_s_gpu"] / osl * unpack_ms / 1e3
                    p = dict(p, tok_s_gpu=p["tok_s_gpu"] / f, tok_s_user=p["tok_s_user"] / f)
                scaled[q].append(p)
        decode = scaled
    for p in agg:
        if p.get("tok_s_user"):
            out["agg"].append({"concurrency": p["concurrency"], "tok_s_gpu": p["tok_s_gpu"], "tok_s_user": p["tok_s_user"],
                               "ttft_p50_ms": p.get("ttft_p50_ms")})
    for q, pts in sorted(decode.items()):
        pts = [p for p in pts if p.get("tok_s_user")]
        pts.sort(key=lambda p: p["concurrency"])
        prev = None
        for p in pts:
            M, u = p["tok_s_gpu"], p["tok_s_user"]
            demand = q * M / osl
            row = {"remote_frac": q, "decode_concurrency": p["concurrency"], "decode_tok_s": M,
                   "tok_s_user": u, "remote_prompts_s": round(demand, 2), "prefill_util": round(demand / prompts_s, 3)}
            if demand <= prompts_s:
                out["disagg"].append({**row, "tok_s_gpu": round(M / 2, 1), "bound": "decode"})
            elif prev is None or q * prev["tok_s_gpu"] / osl <= prompts_s:
                # prefill-bound: the decode GPU settles where the remote demand equals P (below the first
                # measured concurrency: between the origin and it, at that point's tok/s/user -- conservative)
                if prev is None:
                    prev = {"concurrency": 0, "tok_s_gpu": 0.0, "tok_s_user": u}
                d0, d1 = q * prev["tok_s_gpu"] / osl, demand
                f = (prompts_s - d0) / (d1 - d0)
                Mi = prev["tok_s_gpu"] + f * (M - prev["tok_s_gpu"])
                ui = prev["tok_s_user"] + f * (u - prev["tok_s_user"])
                out["disagg"].append({**row, "decode_concurrency": round(prev["concurrency"] + f * (
                    p["concurrency"] - prev["concurrency"]), 1), "decode_tok_s": round(Mi, 1),
                    "tok_s_user": round(ui, 2), "remote_prompts_s": round(prompts_s, 2), "prefill_util": 1.0,
                    "tok_s_gpu": round(Mi / 2, 1), "bound": "prefill"})
            prev = p
    # between two measured remote fractions at one concurrency: the fraction q* at which the remote
    # demand equals P (the conditional policy's queue gate settles there: remote while the prefill
    # GPU keeps up), M and u linear in q between the two sweeps
    qs = sorted(decode)
    for qa, qb in zip(qs, qs[1:]):
        pa = {p["concurrency"]: p for p in decode[qa] if p.get("tok_s_user")}
        pb = {p["concurrency"]: p for p in decode[qb] if p.get("tok_s_user")}
        for c in sorted(set(pa) & set(pb)):
            a, b = pa[c], pb[c]
            da, db = qa * a["tok_s_gpu"] / osl, qb * b["tok_s_gpu"] / osl
            if not da <= prompts_s < db:
                continue
            # demand(q) = q * (Ma + (q - qa) / (qb - qa) * (Mb - Ma)) / osl = P: a quadratic in q
            k = (b["tok_s_gpu"] - a["tok_s_gpu"]) / (qb - qa)
            A, B, C = k, a["tok_s_gpu"] - k * qa, -prompts_s * osl
            if abs(A) < 1e-9:
                q = -C / B
            else:
                disc = B * B - 4 * A * C
                q = max(r for r in ((-B + disc ** 0.5) / (2 * A), (-B - disc ** 0.5) / (2 * A)) if qa - 1e-9 <= r <= qb + 1e-9)
            f = (q - qa) / (qb - qa)
            M = a["tok_s_gpu"] + f * (b["tok_s_gpu"] - a["tok_s_gpu"])
            u = a["tok_s_user"] + f * (b["tok_s_user"] - a["tok_s_user"])
            out["disagg"].append({"remote_frac": round(q, 3), "decode_concurrency": c, "decode_tok_s": round(M, 1),
                                  "tok_s_user": round(u, 2), "remote_prompts_s": round(prompts_s, 2), "prefill_util": 1.0,
                                  "tok_s_gpu": round(M / 2, 1), "bound": "prefill (q interpolated)"})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--agg", required=True, help="bench.py --sweep JSON (aggregated)")
    ap.add_argument("--decode", nargs="+", required=True, help="bench.py --sweep --remote-frac q JSONs")
    ap.add_argument("--prefill-prompts-s", type=float, required=True, help="prefill role: prompts/s at the ISL")
    ap.add_argument("--osl", type=int, default=150)
    ap.add_argument("--isl", type=int, default=3000)
    ap.add_argument("--kv-bytes-per-token", type=int, default=131072,
                    help="KV bytes of one token, all layers (Llama-3-8B bf16: 32 x 2 x 8 x 128 x 2 = 131072; "
                         "70B bf16 327680, fp8 163840)")
    ap.add_argument("--link-GBps", type=float, default=76.5, help="one xGMI link, one direction (0 = no wire charge)")
    ap.add_argument("--pack-overhead", type=float, default=0.007,
                    help="prefill-forward slowdown of the layer-streamed packs (r4_loopback_1p1d.json: 1.007x)")
    ap.add_argument("--unpack-ms", type=float, default=0.1, help="decode-GPU time per remote prompt (unpack)")
    ap.add_argument("--targets", default="20,26,30,40,46,50,60,75,100", help="tok/s/user comparison points")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    _, agg = _load_points(a.agg)
    decode = {}
    for path in a.decode:
        q, pts = _load_points(path)
        decode.setdefault(q, []).extend(pts)
    ch = charged_rates(a.prefill_prompts_s, a.isl, a.kv_bytes_per_token, a.link_GBps, a.pack_overhead, a.unpack_ms)
    res = project(agg, decode, ch["prefill_prompts_s_charged"], a.osl, unpack_ms=a.unpack_ms)
    res["transfer_charge"] = ch
    table = []
    for t in (float(x) for x in a.targets.split(",")):
        ag = frontier([(p["tok_s_user"], p["tok_s_gpu"]) for p in res["agg"]], t)
        dg_pts = [p for p in res["disagg"]]
        dg = frontier([(p["tok_s_user"], p["tok_s_gpu"]) for p in dg_pts], t)
        best = max((p for p in dg_pts if p["tok_s_user"] >= t), key=lambda p: p["tok_s_gpu"], default=None)
        table.append({"tok_s_user": t, "agg_tok_s_gpu": ag and round(ag, 1),
                      "disagg_tok_s_gpu_projected": dg and round(dg, 1),
                      "ratio": round(dg / ag, 3) if ag and dg else None,
                      "best_disagg_point": best and {k: best[k] for k in ("remote_frac", "decode_concurrency", "bound",
                                                                           "prefill_util")}})
    res["prefill_prompts_s"] = a.prefill_prompts_s
    res["osl"] = a.osl
    res["kind"] = "projection from single-GPU role measurements (not a multi-GPU measurement)"
    res["table"] = table
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)
    print(f"# PROJECTED, transfer charged: wire {ch['wire_ms']} ms per prompt ({ch['kv_mb_per_prompt']} MB over one "
          f"{a.link_GBps} GB/s link), pack +{a.pack_overhead * 100:.1f} %, unpack {a.unpack_ms} ms: prefill GPU "
          f"{a.prefill_prompts_s:.2f} -> {ch['prefill_prompts_s_charged']:.2f} prompts/s")
    print(f"{'tok/s/user':>10} {'agg tok/s/GPU':>14} {'xPyD (proj.)':>15} {'ratio':>6}  best disagg point")
    for r in table:
        print(f"{r['tok_s_user']:>10} {r['agg_tok_s_gpu'] or '-':>14} {r['disagg_tok_s_gpu_projected'] or '-':>15} "
              f"{r['ratio'] or '-':>6}  {r['best_disagg_point']}")
    return res


if __name__ == "__main__":
    main()
