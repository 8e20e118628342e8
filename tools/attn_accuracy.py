"""Prefill-attention accuracy of the kernel variants (ops.PREFILL_WAVES 91 /
92) against an fp32 reference of the same op, on random data at a few
shapes: max and mean absolute error, and the error relative to |ref|."""
import math
import sys

import torch

sys.path.insert(0, ".")
from dynamo_exp_amd import ops  # noqa: E402
from dynamo_exp_amd.ops import reference as ref  # noqa: E402

torch.manual_seed(0)
for L, nseq, scale_q in ((700, 3, 1.0), (2000, 1, 1.0), (1500, 2, 4.0)):
    Hq, Hkv, D, bs = 32, 8, 128, 64
    nb = nseq * (L // bs + 1) + 4
    kc = torch.randn(nb, Hkv, bs, D, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.arange(nb - 4, dtype=torch.int32).view(nseq, -1)
    q = (torch.randn(nseq * L, Hq, D) * scale_q).to(torch.bfloat16)
    cu = torch.arange(0, nseq * L + 1, L, dtype=torch.int32)
    ctx = torch.full((nseq,), L, dtype=torch.int32)
    want = ref.paged_attention(q.float(), kc.float(), vc.float(), bt, cu, ctx, 1 / math.sqrt(D), bs).float()
    row = {}
    for v in (92, 91):
        ops.PREFILL_WAVES = v
        out = torch.empty(q.shape, dtype=torch.bfloat16, device="cuda")
        ops.prefill_attention(q.cuda(), kc.cuda(), vc.cuda(), bt.cuda(), cu.cuda(), ctx.cuda(), 1 / math.sqrt(D), out)
        e = (out.float().cpu() - want).abs()
        row[v] = (round(e.max().item(), 5), round(e.mean().item(), 6))
    print(f"L{L}x{nseq} q*{scale_q}: max / mean abs error vs fp32 -- 92 {row[92]}, 91 {row[91]}; |ref| mean "
          f"{want.abs().mean().item():.4f}", flush=True)
