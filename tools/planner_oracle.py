#!/usr/bin/env python3
"""What ANY planner could achieve on the planner benchmark's regime: a
clairvoyant lower bound.

The benchmark (tools/planner_bench.py --slowdown 3.5 --gpu-gb 80): Poisson
arrivals at rate(t) = 12.5 + 7.5 sin(2 pi t / 150) req/s for 600 s, ISL 3000 /
OSL 150, sim workers = engine/sim.py's MI355X timing model of Llama-3-8B TP1
made 3.5x slower.  The reference's result (8x H100,
docs/guides/planner_benchmark/benchmark_planner.md:20-35): the planner beat
static 2P2D by 33 % average latency AND 7.6 % GPU-seconds.

Fluid model with every assumption in the planner's favour:
* scaling is instant and free (no start-up, no drain, no adjustment interval:
  the pool can change every second), and clairvoyant (the rate is known);
* prefill: a prompt costs ISL / prefill rate of one worker; with P workers the
  TTFT is that service time alone while rate <= P x capacity (no queueing at
  all -- a real M/D/P queue waits longer), and the oracle never overloads;
* decode: deterministic fluid steps, step = decode_ms + per_seq x streams per
  worker + host_ms, the streams in decode from Little's law
  (N = rate x OSL x step), so ITL = (decode_ms + host_ms) / (1 - rate x OSL x
  per_seq / D).
Per second it picks (P, D) minimising P + D + mu x rate x latency; scanning mu
traces the best GPU-seconds for each request-weighted mean latency.  Static
2P2D runs through the same model (a prefill backlog builds while rate > 2 x
capacity) to show how close the model is to the measured run.

    python tools/planner_oracle.py [--out profiles/r6_planner_oracle.json]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def model_params(slowdown: float) -> dict:
    """The sim engine's timing constants (engine/sim.py SimLLMEngine.mi355x_8b)."""
    from dynamo_exp_amd.engine.sim import SimLLMEngine

    d = SimLLMEngine.mi355x_8b("decode", slowdown=slowdown, gpu_gb=80.0)
    p = SimLLMEngine.mi355x_8b("prefill", slowdown=slowdown, gpu_gb=80.0)
    return {"decode_ms": d.decode_ms, "per_seq_ms": d.decode_per_seq_ms, "host_ms": d.host_ms,
            "prefill_tok_per_ms": p.prefill_tok_per_ms, "decode_slots": d.max_num_seqs}


def itl_ms(rate: float, D: int, osl: int, m: dict) -> float | None:
    a = m["decode_ms"] + m["host_ms"]
    x = rate * osl * m["per_seq_ms"] / 1e3 / D
    if x >= 1.0:
        return None
    itl = a / (1.0 - x)
    if rate * osl * itl / 1e3 / D > m["decode_slots"]:
        return None
    return itl


def slot_latency(rate: float, P: int, D: int, isl: int, osl: int, m: dict) -> float | None:
    """Latency (s) of a request arriving at `rate` with P / D workers (no queueing)."""
    svc = isl / m["prefill_tok_per_ms"] / 1e3
    if rate * svc >= P:  # the oracle never overloads its prefill pool
        return None
    itl = itl_ms(rate, D, osl, m)
    return None if itl is None else svc + osl * itl / 1e3


def oracle(rates: list[float], isl: int, osl: int, m: dict, mu: float, max_gpus: int = 8) -> tuple[float, float]:
    """(request-weighted mean latency, GPU-seconds) of the per-second optimum for multiplier mu."""
    lat_w = gpu = req = 0.0
    for r in rates:
        best = None
        for P in range(1, max_gpus):
            for D in range(1, max_gpus - P + 1):
                lat = slot_latency(r, P, D, isl, osl, m)
                if lat is None:
                    continue
                c = P + D + mu * r * lat
                if best is None or c < best[0]:
                    best = (c, P, D, lat)
        if best is None:
            raise RuntimeError(f"rate {r}: no feasible pool within {max_gpus} GPUs")
        _, P, D, lat = best
        gpu += P + D
        lat_w += r * lat
        req += r
    return lat_w / req, gpu


def static(rates: list[float], P: int, D: int, isl: int, osl: int, m: dict) -> tuple[float, float]:
    """Static pool, fluid prefill backlog (FIFO): TTFT = service + backlog / capacity."""
    svc = isl / m["prefill_tok_per_ms"] / 1e3
    cap = P / svc  # prompts/s
    q = lat_w = req = 0.0
    for _ in range(3):  # settle the periodic backlog
        q0 = q
        lat_w = req = 0.0
        for r in rates:
            q = max(0.0, q + r - cap)
            itl = itl_ms(min(r, cap), D, osl, m)
            lat = svc + q / cap + osl * itl / 1e3
            lat_w += r * lat
            req += r
        if abs(q - q0) < 1e-6:
            break
    return lat_w / req, (P + D) * len(rates)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--slowdown", type=float, default=3.5)
    ap.add_argument("--min-rate", type=float, default=5.0)
    ap.add_argument("--max-rate", type=float, default=20.0)
    ap.add_argument("--period", type=float, default=150.0)
    ap.add_argument("--duration", type=float, default=600.0)
    ap.add_argument("--isl", type=int, default=3000)
    ap.add_argument("--osl", type=int, default=150)
    ap.add_argument("--measured-static-latency", type=float, default=7.512,
                    help="static 2P2D measured on the benchmark (profiles/r5_planner_overload_static_2p2d.json)")
    ap.add_argument("--measured-static-gpu-s", type=float, default=2415.5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    m = model_params(a.slowdown)
    mid, amp = (a.max_rate + a.min_rate) / 2, (a.max_rate - a.min_rate) / 2
    rates = [mid + amp * math.sin(2 * math.pi * (t + 0.5) / a.period) for t in range(int(a.duration))]
    s_lat, s_gpu = static(rates, 2, 2, a.isl, a.osl, m)
    front = []
    for mu in [0.0] + [10 ** (k / 8) for k in range(-24, 25)]:
        lat, gpu = oracle(rates, a.isl, a.osl, m, mu)
        front.append({"mu": mu, "latency_s": round(lat, 3), "gpu_s": round(gpu, 1)})
    ref_lat = a.measured_static_latency * (1 - 0.33)
    ref_gpu = a.measured_static_gpu_s * (1 - 0.076)
    # the cheapest oracle point at or below the latency target
    ok = [p for p in front if p["latency_s"] <= ref_lat]
    best = min(ok, key=lambda p: p["gpu_s"]) if ok else None
    res = {"model": m, "trace": {"min_rate": a.min_rate, "max_rate": a.max_rate, "period": a.period,
                                 "duration": a.duration, "isl": a.isl, "osl": a.osl},
           "static_2p2d_model": {"latency_s": round(s_lat, 3), "gpu_s": s_gpu},
           "static_2p2d_measured": {"latency_s": a.measured_static_latency, "gpu_s": a.measured_static_gpu_s},
           "reference_relative_target": {"latency_s": round(ref_lat, 3), "gpu_s": round(ref_gpu, 1)},
           "oracle_frontier": front,
           "oracle_at_target_latency": best,
           "verdict": None}
    if best is None:
        res["verdict"] = "no pool schedule reaches the latency target in this model"
    else:
        res["verdict"] = (f"the clairvoyant, instant-scaling oracle needs {best['gpu_s']:.0f} GPU-s for "
                          f"{best['latency_s']:.2f} s mean latency (target {ref_lat:.2f} s, <= {ref_gpu:.0f} GPU-s): "
                          + ("feasible" if best["gpu_s"] <= ref_gpu else "INFEASIBLE for any planner"))
    print(json.dumps({k: v for k, v in res.items() if k != "oracle_frontier"}, indent=1))
    for p in front[::4]:
        print(f"  mu {p['mu']:<10.4g} latency {p['latency_s']:6.3f} s  GPU-s {p['gpu_s']:7.1f}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return res


if __name__ == "__main__":
    main()
