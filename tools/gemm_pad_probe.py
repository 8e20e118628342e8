"""Prefill projections (qkv / o / down, hipBLASLt via torch.matmul) at the
token counts a mixed step has: time at M, at M padded up to the next multiple
of 256, and the hand 256x256 kernel (gemm256, store epilogue) at M; weights
rotated over 8 copies.  Decides whether to pad / reroute (models/llama.py).

  python -m tools.gemm_pad_probe
"""
import json

import torch

from dynamo_exp_amd import ops
from tools.gemm_bench import timed


def main():
    H, F = 4096, 14336
    ws = {"qkv": [torch.randn(6144, H, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(8)],
          "o": [torch.randn(H, H, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(8)],
          "down": [torch.randn(H, F, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(8)]}
    res = {}
    for b in range(1024, 8193, 512):
        for M in (b - 200, b - 40, b):
            row = {}
            for name, wl in ws.items():
                N, K = wl[0].shape
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                xp = torch.zeros(-(-M // 256) * 256, K, device="cuda", dtype=torch.bfloat16)
                t_lib = timed(lambda: [torch.matmul(x, w.t()) for w in wl], 3) / len(wl)
                t_pad = timed(lambda: [torch.matmul(xp, w.t()) for w in wl], 3) / len(wl)
                t_g = timed(lambda: [ops.gemm256(x, w) for w in wl], 3) / len(wl)
                row[name] = (round(t_lib, 1), round(t_pad, 1), round(t_g, 1))
            res[M] = row
            print(f"M {M}: us (lib, lib@pad256, gemm256) {row}", flush=True)
    with open("gpurun_out/gemm_pad_probe.json", "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
