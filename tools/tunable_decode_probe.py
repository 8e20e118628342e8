"""Does PyTorch TunableOp (exhaustive hipBLASLt / rocBLAS solution search) find
faster solutions than hipBLASLt's default heuristic at the DECODE projection
shapes (M = decode batch 64-256)?  Weights cold (rotating over 32 copies), as
in a real decode step.  (The prefill-shape study is r1_gemm_tunableop_study.txt.)

  python tools/tunable_decode_probe.py --out gpurun_out/tunable_decode.json
"""
import argparse
import json
import os
import time

import torch

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
    ap.add_argument("--out", default="gpurun_out/tunable_decode.json")
    ap.add_argument("--ms", default="64,128,256")
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--csv", default="gpurun_out/tunableop_decode.csv")
    a = ap.parse_args()
    tun = torch.cuda.tunable
    tun.set_filename(a.csv)
    tun.set_max_tuning_duration(30)
    tun.set_max_tuning_iterations(20)
    tun.set_rotating_buffer_size(512)  # MB: tune with cold operands
    res = {}
    for name, (N, K) in SHAPES.items():
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(a.copies)]
        gb = N * K * 2 / 1e9
        for M in map(int, a.ms.split(",")):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            tun.enable(False)
            lib = timed(lambda: [torch.matmul(x, w.t()) for w in ws]) / len(ws)
            tun.enable(True)
            tun.tuning_enable(True)
            t0 = time.time()
            torch.matmul(x, ws[0].t())
            torch.cuda.synchronize()
            tune_s = time.time() - t0
            tun.tuning_enable(False)
            tuned = timed(lambda: [torch.matmul(x, w.t()) for w in ws]) / len(ws)
            want = (x.float() @ ws[0].float().t())
            err = ((torch.matmul(x, ws[0].t()).float() - want).abs().max() / want.abs().max()).item()
            tun.enable(False)
            r = {"lib_us": round(lib, 1), "lib_TBs": round(gb / lib * 1e3, 2), "tuned_us": round(tuned, 1),
                 "tuned_TBs": round(gb / tuned * 1e3, 2), "speedup": round(lib / tuned, 2), "tune_s": round(tune_s, 1),
                 "rel_err": err}
            res[f"{name}_M{M}"] = r
            print(name, M, r, flush=True)
        del ws
        torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
