"""Decode attention bf16 vs fp8 KV (B 128, ~3100 context), 20 launches each --
the program a rocprofv3 --pmc pass wraps (tools/pmc_summary.py reads it)."""
import math

import torch

from dynamo_exp_amd import ops


def main():
    Hq, Hkv, D, bs, B, L = 32, 8, 128, 64, 128, 3100
    nbps = L // bs + 1
    kc = torch.randn(B * nbps, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    k8, v8 = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
    bt = torch.randperm(B * nbps, device="cuda").to(torch.int32).view(B, nbps)
    q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
    ctx = torch.randint(L - 150, L, (B,), dtype=torch.int32, device="cuda")
    out = torch.empty_like(q)
    mp = ops.decode_num_parts(B, Hkv, L)
    ws = ops.decode_workspace(B, Hq, D, mp, "cuda")
    for kk, vv in ((kc, vc), (k8, v8)):
        for _ in range(20):
            ops.decode_attention(q, kk, vv, bt, ctx, 1 / math.sqrt(D), out, mp, workspace=ws)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
