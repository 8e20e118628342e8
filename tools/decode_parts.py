"""Decode attention: HBM rate vs number of balanced partitions per sequence
(ops.decode_num_parts picks the default)."""
import json, math, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamo_exp_amd import ops
from tools.microbench import bench

Hq, Hkv, D, bs = 32, 8, 128, 64
res = {}
for B, L in ((64, 3072), (128, 3072), (128, 3100), (256, 3100), (16, 8000)):
    nbps = L // bs + 1
    nb = B * nbps
    kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.randperm(nb, device="cuda").to(torch.int32).view(B, nbps)
    q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
    ctx = torch.full((B,), L, dtype=torch.int32, device="cuda")
    out = torch.empty_like(q)
    row = {}
    for P in (1, 2, 3, 4, 6, 8, 12, 16):
        ws = ops.decode_workspace(B, Hq, D, P, "cuda")
        us = bench(lambda: ops.decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out, P, workspace=ws), 30)
        row[P] = round(B * L * Hkv * D * 4 / us / 1e6, 2)
    res[f"B{B}_L{L} (default P={ops.decode_num_parts(B, Hkv, L)})"] = row
    del kc, vc
print(json.dumps(res, indent=0))
