#!/usr/bin/env python3
"""Decode-projection GEMM sweep on one MI355X: hipBLASLt vs the deep-stream
kernel (csrc/kernels/dstream_gemm.hip) over every valid configuration, for
the Llama-3-8B TP1 projections at decode batch sizes.  Weights: L distinct
per-layer copies, timed in turn (their footprint is far beyond the 256 MB
Infinity Cache, so every call streams from HBM as in a decode step).  The
best configuration per shape is checked against torch.matmul.

    python tools/dstream_bench.py --out profiles/r4_dstream_sweep.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="64,128,256")
    ap.add_argument("--layers", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch

    from dynamo_exp_amd import ops

    dev = torch.device("cuda:0")
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}

    def timed(fn) -> float:
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps

    res = {}
    for name in a.shapes.split(","):
        N, K = shapes[name]
        nl = max(2, min(a.layers, int(6e9 // (N * K * 2))))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nl)]
        wbytes = N * K * 2
        for M in [int(m) for m in a.m.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            lib = timed(lambda: [torch.matmul(x, w.t()) for w in ws]) / nl
            rows = []
            for cfg in ops.dstream_configs(M, N, K):
                try:
                    t = timed(lambda: [ops.dstream_linear(x, w, cfg) for w in ws]) / nl
                except Exception as e:  # noqa: BLE001
                    rows.append((1e9, cfg, repr(e)))
                    continue
                rows.append((t, cfg, None))
            rows.sort(key=lambda r: r[0])
            best = rows[0]
            want = torch.matmul(x, ws[0].t()).float()
            got = ops.dstream_linear(x, ws[0], best[1]).float()
            err = ((got - want).abs().max() / want.abs().max()).item()
            key = f"{name}_M{M}"
            res[key] = {"N": N, "K": K, "M": M, "lib_us": round(lib, 2), "lib_TBs": round(wbytes / lib / 1e6, 2),
                        "best_us": round(best[0], 2), "best_TBs": round(wbytes / best[0] / 1e6, 2),
                        "best_cfg": best[1], "rel_err": err, "speedup": round(lib / best[0], 3),
                        "top": [[round(t, 2), c] for t, c, _ in rows[:a.top]],
                        "errors": [[c, e] for _, c, e in rows if e][:3]}
            print(json.dumps({k: res[key][k] for k in ("lib_us", "lib_TBs", "best_us", "best_TBs", "best_cfg",
                                                         "rel_err", "speedup")} | {"shape": key}), flush=True)
        del ws
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
