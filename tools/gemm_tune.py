"""GEMM solution study for the Llama-3-8B serving shapes on MI355X.

Measures hipBLASLt's default heuristic pick vs PyTorch TunableOp (exhaustive
hipBLASLt + rocBLAS solution search per shape), and writes the tuned table so
the engine can load it (`DX_GEMM_TUNED=<csv>`).

  python tools/gemm_tune.py --out gpurun_out/gemm_tune.json --csv gpurun_out/tunableop.csv
"""
from __future__ import annotations

import argparse
import json

import torch

H, F = 4096, 14336
LAYERS = {"qkv": (H, 6144), "o": (H, H), "gate_up": (H, 2 * F), "down": (F, H)}


def bench(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def run_all(Ms, tag, res):
    for M in Ms:
        for name, (K, N) in LAYERS.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            us = bench(lambda: torch.matmul(x, w.t()), iters=10 if M >= 4096 else 50)
            res.setdefault(f"{name}_M{M}", {})[tag] = {"us": round(us, 1),
                                                       "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}
            print(name, M, tag, res[f"{name}_M{M}"][tag], flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/gemm_tune.json")
    ap.add_argument("--csv", default="gpurun_out/tunableop.csv")
    ap.add_argument("--M", default="16384,8192,3072,256,128,64")
    ap.add_argument("--tune-ms", type=int, default=30)
    a = ap.parse_args()
    Ms = [int(m) for m in a.M.split(",")]
    res = {}
    run_all(Ms, "default", res)
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(a.tune_ms)
    tun.set_filename(a.csv)
    run_all(Ms, "tuned", res)
    tun.tuning_enable(False)
    run_all(Ms, "tuned_replay", res)
    json.dump(res, open(a.out, "w"), indent=1)  # the tuned CSV is flushed at exit


if __name__ == "__main__":
    main()
