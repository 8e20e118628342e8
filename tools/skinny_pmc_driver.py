"""Tiny driver for rocprofv3 --pmc runs on the small-M GEMM: the wide kernel
(cfg 128, 128, s) and the narrow kernel at the Llama-3-8B decode shapes, M 128,
cold weights (8 rotating copies), 10 launches each.

  rocprofv3 --kernel-trace --pmc <counters> -- python3 tools/skinny_pmc_driver.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dynamo_exp_amd import ops  # noqa: E402

CASES = [("gate_up", 28672, 4096, (128, 128, 1)), ("down", 4096, 14336, (128, 128, 8)),
         ("qkv", 6144, 4096, (64, 64, 1)), ("qkv_wide", 6144, 4096, (128, 128, 4))]


def main():
    M = 128
    for name, N, K, cfg in CASES:
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(8)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        for i in range(10):
            ops.skinny_linear(x, ws[i % 8], cfg)
        torch.cuda.synchronize()
        print(name, cfg, "done", flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
