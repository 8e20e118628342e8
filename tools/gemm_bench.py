"""Prefill-GEMM microbench: the hand-written 256x256 MFMA GEMM
(csrc/kernels/gemm256.hip) vs hipBLASLt (torch.matmul) at the Llama-3-8B
projection shapes, and the fused SwiGLU epilogue vs hipBLASLt gate_up +
silu_and_mul.  Uniform random operands (guide §5.4 rule 25), weights rotated
over enough copies to exceed the 256 MB Infinity Cache, interleaved rounds in
one process (rule 24).  Prints one JSON object."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamo_exp_amd import ops  # noqa: E402
from dynamo_exp_amd.ops import reference as ref  # noqa: E402


def timed(fn, iters):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[3000, 8192])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=8)
    a = ap.parse_args()
    dev = "cuda"
    H, F = 4096, 14336
    shapes = {"qkv": (6144, H), "o": (H, H), "gate_up": (2 * F, H), "down": (H, F)}
    res = {}
    for M in a.m:
        x = {K: (torch.rand(M, K, device=dev) * 2 - 1).bfloat16() for K in (H, F)}
        for name, (N, K) in shapes.items():
            copies = max(2, int(600e6 // (N * K * 2)))
            ws = [(torch.rand(N, K, device=dev) * 2 - 1).bfloat16().mul_(K ** -0.5) for _ in range(copies)]
            it = [0]

            def nxt():
                it[0] += 1
                return ws[it[0] % copies]

            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            arms = {"hipblaslt": lambda: torch.matmul(x[K], nxt().t(), out=out),
                    "gemm256": lambda: ops.gemm256(x[K], nxt(), out=out),
                    "gemm256_1tile": lambda: ops.gemm256(x[K], nxt(), out=out, group_m=1008)}
            if name == "gate_up":
                wis = [ref.interleave_gate_up(w, ops.GEMM256_BLK).contiguous() for w in ws]
                act = torch.empty(M, F, device=dev, dtype=torch.bfloat16)

                def nxti():
                    it[0] += 1
                    return wis[it[0] % copies]

                arms["hipblaslt+silu"] = lambda: ops.silu_and_mul(torch.matmul(x[K], nxt().t(), out=out), out=act)
                arms["fused_silu"] = lambda: ops.gemm256(x[K], nxti(), ops.GEMM256_EPI_SILU, out=act)
                arms["fused_silu_1tile"] = lambda: ops.gemm256(x[K], nxti(), ops.GEMM256_EPI_SILU, out=act,
                                                               group_m=1008)
            tms = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, fn in arms.items():
                    tms[k].append(timed(fn, a.iters))
            flop = 2.0 * M * N * K
            row = {}
            for k, v in tms.items():
                v.sort()
                row[k] = {"us_med": round(v[len(v) // 2], 1), "us_min": round(v[0], 1),
                          "tflops_med": round(flop / v[len(v) // 2] / 1e6, 1)}
            res[f"M{M}_{name}"] = row
            print(f"M={M} {name}: " + ", ".join(f"{k} {r['us_med']}us {r['tflops_med']}TF" for k, r in row.items()),
                  file=sys.stderr, flush=True)
            del ws
            torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
