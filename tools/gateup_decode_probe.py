#!/usr/bin/env python3
"""Decode-size gate_up + SwiGLU: is the 256x256-tile fused kernel (gemm256,
EPI_SILU) competitive with hipBLASLt + silu_and_mul at M 64-256?

At M = 128 the decode step's gate_up (N 28672, K 4096, 235 MB of weights) runs
on hipBLASLt at ~4.4 TB/s (profiles/r6_decode_gemm_report.json); gemm256 puts
one 256-token tile x 112 weight tiles on 112 CUs, each streaming 2 MB of
weights, with the activation fused.  Times every candidate with HIP events
over 50 repetitions after warm-up, one row per M, and checks the fused output
against the library path.

    python tools/gateup_decode_probe.py [--out gpurun_out/gateup_decode_probe.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    import torch

    from dynamo_exp_amd import ops
    from dynamo_exp_amd.ops import reference as ref

    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args(argv)
    dev = torch.device("cuda:0")
    K, F = 4096, 14336
    torch.manual_seed(0)
    w = (torch.randn(2 * F, K, device=dev) / 64).bfloat16()
    wi = ref.interleave_gate_up(w, ops.GEMM256_BLK).contiguous()
    wbytes = wi.numel() * 2

    def timed(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3 / a.reps  # us

    rows = []
    for M in (32, 64, 96, 128, 160, 192, 256, 384):
        x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        lib = timed(lambda: ops.silu_and_mul(torch.matmul(x, wi.t()), blk=ops.GEMM256_BLK))
        fused = {}
        for gm in (1, 2, 8):
            fused[gm] = timed(lambda gm=gm: ops.gemm256(x, wi, ops.GEMM256_EPI_SILU, group_m=gm))
        got = ops.gemm256(x, wi, ops.GEMM256_EPI_SILU)
        want = ops.silu_and_mul(torch.matmul(x, wi.t()), blk=ops.GEMM256_BLK)
        err = ((got.float() - want.float()).abs().max() / want.float().abs().max()).item()
        best = min(fused, key=fused.get)
        r = {"M": M, "lib_silu_us": round(lib, 2), "gemm256_us": {k: round(v, 2) for k, v in fused.items()},
             "best_gm": best, "speedup": round(lib / fused[best], 3),
             "gemm256_TBps": round(wbytes / fused[best] / 1e6, 2), "lib_TBps": round(wbytes / lib / 1e6, 2),
             "rel_err": round(err, 5)}
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
