"""Bandwidth probe of the weight-streaming GEMM (csrc/kernels/wstream_gemm.hip):
times one config with the x DMA and / or the MFMAs switched off (wpol bits 1 / 2;
the results are wrong in those modes), weights cold over 32 copies.

  python -m tools.wstream_probe
"""
import torch

from dynamo_exp_amd import ops
from tools.skinny_bench import SHAPES, timed


def main():
    cases = [("down", 128, ("ws", 128, 64, 4, 4, 64)), ("gate_up", 128, ("ws", 128, 128, 4, 1, 64)),
             ("down", 128, ("ws", 128, 128, 3, 4, 64)), ("qkv", 128, ("ws", 128, 64, 4, 2, 64))]
    for name, M, cfg in cases:
        N, K = SHAPES[name]
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(32)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        gb = N * K * 2 / 1e9
        row = {}
        for mode, bits in (("full", 0), ("nt", 1), ("no_x", 2), ("no_mfma", 4), ("dma_w_only", 6)):
            t = timed(lambda: [ops.skinny_linear(x, w, cfg + (bits,)) for w in ws]) / len(ws)
            row[mode] = f"{t:.1f}us {gb / t * 1e3:.2f}TB/s"
        print(name, M, cfg, row, flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
