"""Bandwidth probe of the weight-streaming GEMM (csrc/kernels/wstream_gemm.hip):
times one config with the x DMA and / or the MFMAs switched off (wpol bits 1 / 2;
the results are wrong in those modes), weights cold over 32 copies.

  python -m tools.wstream_probe
"""
import torch

from dynamo_exp_amd import ops
from tools.skinny_bench import SHAPES, timed


HOT = False


def main():
    global HOT
    import sys
    HOT = "--hot" in sys.argv
    cases = [(n, 128, ("ws", 128, bn, 4, s, 64, nw)) for n, bn, s in (("down", 64, 4), ("gate_up", 128, 1), ("qkv", 64, 2))
             for nw in (4, 8)]
    for name, M, cfg in cases:
        N, K = SHAPES[name]
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(32)]
        if HOT:  # one copy, re-read: served by the 256 MB Infinity Cache (MALL)
            ws = [ws[0]] * 32
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        gb = N * K * 2 / 1e9
        row = {"hipblaslt": f"{timed(lambda: [torch.matmul(x, w.t()) for w in ws]) / len(ws):.1f}us"}
        for mode, bits in (("full", 0), ("nt", 1), ("no_mfma", 4), ("dma_w_only", 6), ("blocked_w", 8)):
            t = timed(lambda: [ops.skinny_linear(x, w, cfg + (bits,)) for w in ws]) / len(ws)
            row[mode] = f"{t:.1f}us {gb / t * 1e3:.2f}TB/s"
        print(name, M, cfg, row, flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
