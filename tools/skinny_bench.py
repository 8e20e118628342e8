"""Small-M GEMM sweep: hipBLASLt vs every launch config of the hand-written
MFMA kernels (csrc/kernels/skinny_gemm.hip, dstream_gemm.hip) at the Llama-3-8B projection shapes,
weights cold (rotating over 32 copies, > the 256 MB Infinity Cache, as in a
real decode step).

  python tools/skinny_bench.py --out gpurun_out/skinny.json
"""
import argparse
import json

import torch

from dynamo_exp_amd import ops

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timed(fn, reps=3):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/skinny.json")
    ap.add_argument("--ms", default="16,64,128,256")
    ap.add_argument("--copies", type=int, default=32)
    a = ap.parse_args()
    res = {}
    for name, (N, K) in SHAPES.items():
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(a.copies)]
        gb = N * K * 2 / 1e9
        for M in map(int, a.ms.split(",")):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            lib = timed(lambda: [torch.matmul(x, w.t()) for w in ws]) / len(ws)
            rows = []
            for cfg in ops.skinny_configs(M, N, K) + ops.dstream_configs(M, N, K):
                t = timed(lambda: [ops.skinny_linear(x, w, cfg) for w in ws]) / len(ws)
                rows.append((t, cfg))
            rows.sort()
            best_t, best_cfg = rows[0]
            r = {"lib_us": round(lib, 1), "lib_TBs": round(gb / lib * 1e3, 2), "best_us": round(best_t, 1),
                 "best_TBs": round(gb / best_t * 1e3, 2), "best_cfg": best_cfg, "speedup": round(lib / best_t, 2),
                 "top3": [(round(t, 1), c) for t, c in rows[:3]]}
            res[f"{name}_M{M}"] = r
            print(name, M, r, flush=True)
        del ws
        torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
