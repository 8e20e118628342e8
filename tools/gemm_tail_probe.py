"""Wave quantization of the prefill GEMMs over the token counts a mixed step
actually has: TFLOP/s of the fused SwiGLU gemm256 (gate_up) and of hipBLASLt
(qkv / o / down) at M from 1024 to 8320, weights rotated over 8 copies.

  python -m tools.gemm_tail_probe
"""
import torch

from dynamo_exp_amd import ops
from tools.gemm_bench import timed


def main():
    H, F = 4096, 14336
    ws = {"gate_up": [torch.randn(2 * F, H, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(8)],
          "qkv": [torch.randn(6144, H, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(8)],
          "o": [torch.randn(H, H, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(8)],
          "down": [torch.randn(H, F, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(8)]}
    for M in (1064, 2048, 3072, 4096, 4864, 5120, 5736, 6144, 7168, 7936, 8192, 8320):
        row = {}
        for name, wl in ws.items():
            N, K = wl[0].shape
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            if name == "gate_up":
                fn = lambda: [ops.gemm256(x, w, ops.GEMM256_EPI_SILU) for w in wl]
            else:
                fn = lambda: [torch.matmul(x, w.t()) for w in wl]
            us = timed(fn, 3) / len(wl)
            row[name] = round(2 * M * N * K / us / 1e6, 0)
        print(f"M {M}: TFLOP/s {row}", flush=True)


if __name__ == "__main__":
    main()
