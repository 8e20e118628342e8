"""Which shapes of the decode-attention kernel produce NaN (debug probe)."""
import math
import sys

import torch

sys.path.insert(0, ".")
from dynamo_exp_amd import ops  # noqa: E402
from dynamo_exp_amd.ops import reference as ref  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
for hq, hkv in ((8, 8), (16, 8), (32, 8), (16, 2)):
    for bs in (16, 64):
        for L in (1, 17, 64, 333):
            nb = (L + bs - 1) // bs + 1
            kc = torch.randn(nb, hkv, bs, 128, device=dev, dtype=torch.bfloat16)
            vc = torch.randn_like(kc)
            bt = torch.arange(nb, dtype=torch.int32, device=dev).view(1, -1)
            q = torch.randn(1, hq, 128, device=dev, dtype=torch.bfloat16)
            ctx = torch.tensor([L], dtype=torch.int32, device=dev)
            out = torch.empty_like(q)
            ops.decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(128), out, 1)
            exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), torch.arange(2, dtype=torch.int32),
                                      ctx.cpu(), 1 / math.sqrt(128), bs)
            o = out.float().cpu()
            nan = torch.isnan(o)
            print(hq, hkv, bs, L, "nan heads/dims:", int(nan.any(-1).sum()), int(nan.any(1).sum()),
                  "max err", float((o - exp.float()).abs().nan_to_num(99).max()), flush=True)
