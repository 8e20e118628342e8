#!/usr/bin/env python3
"""Where the deep-stream decode GEMM's time goes (csrc/kernels/dstream_gemm.hip
probe modes, config nw 4 / r 1 / t 8 / dw 4 / dx 4 at M 128): 0 = the GEMM,
1 = no LDS reads / MFMA, 2 = also no x DMA (weights + per-step barrier),
3 = weights only.  Same grids and weight copies as the GEMM timings.

    python tools/dstream_probe.py --out profiles/r4_dstream_probe.txt
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from dynamo_exp_amd import ops

    dev = torch.device("cuda:0")
    k = ops._k()
    lines = []
    for name, N, K, splits in (("qkv", 6144, 4096, 2), ("qkv", 6144, 4096, 4), ("o", 4096, 4096, 4),
                               ("gate_up", 28672, 4096, 1), ("down", 4096, 14336, 4)):
        nl = max(2, min(16, int(4e9 // (N * K * 2))))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nl)]
        x = torch.randn(128, K, device=dev, dtype=torch.bfloat16)
        y = torch.empty(128, N, device=dev, dtype=torch.bfloat16)
        st = ops._stream()
        slabs, tickets = ops._skinny_ws(dev, st)
        res = {}
        for p in (0, 1, 2, 3):
            def run():
                for w in ws:
                    k.dstream_probe(y.data_ptr(), y.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(),
                                    slabs.data_ptr(), tickets.data_ptr(), 128, N, K, splits, p, st)
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                run()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 3 / nl
            res[p] = f"{us:.1f}us {N * K * 2 / us / 1e6:.2f}TB/s"
        line = f"{name} M128 splits {splits} grid {N // 64 * splits}: " + ", ".join(
            f"{('gemm', 'no_compute', 'w+barrier', 'w_only')[p]} {v}" for p, v in res.items())
        print(line, flush=True)
        lines.append(line)
        del ws
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
