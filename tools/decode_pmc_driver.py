"""Decode attention under rocprofv3 --pmc (tools/pmc_summary.py reads the counter CSV): B 128, ~3100-token
contexts, bf16 and fp8 caches, the MFMA kernel and the VALU kernel (DX_DECODE_MFMA is read per call; the two are
different kernel names in the CSV), at 32 q / 8 kv heads (Llama-3-8B) and 16 / 2 (one Llama-3-70B TP4 rank);
20 launches each."""
import math
import os

import torch

from dynamo_exp_amd import ops


def main():
    D, bs, B, L = 128, 64, 128, 3100
    nbps = L // bs + 1
    for Hq, Hkv in ((32, 8), (16, 2)):
        kc = torch.randn(B * nbps, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        k8, v8 = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
        bt = torch.randperm(B * nbps, device="cuda").to(torch.int32).view(B, nbps)
        q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
        ctx = torch.randint(L - 150, L, (B,), dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        mp = ops.decode_num_parts(B, Hkv, L)
        ws = ops.decode_workspace(B, Hq, D, mp, "cuda")
        for mf in ("1", "0"):
            os.environ["DX_DECODE_MFMA"] = mf
            for kk, vv in ((kc, vc), (k8, v8)):
                for _ in range(20):
                    ops.decode_attention(q, kk, vv, bt, ctx, 1 / math.sqrt(D), out, mp, workspace=ws)
            torch.cuda.synchronize()
        del kc, vc, k8, v8
    os.environ.pop("DX_DECODE_MFMA", None)


if __name__ == "__main__":
    main()
