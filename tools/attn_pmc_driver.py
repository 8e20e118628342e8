"""Workload for rocprofv3 --pmc passes over the prefill-attention kernel:
the round-3 loop (ops.PREFILL_WAVES 92) and the current one (91) at the
headline shapes (5 x 3000 and 1 x 16000, causal, paged KV, block 64), a few
launches each; the two variants are different template instances, so the
counter CSV separates them by kernel name.

  rocprofv3 --pmc ... -- python3 -m tools.attn_pmc_driver
"""
import math
import sys

import torch

sys.path.insert(0, ".")
from dynamo_exp_amd import ops  # noqa: E402


def main():
    Hq, Hkv, D, bs = 32, 8, 128, 64
    for L, nseq in ((3000, 5), (16000, 1)):
        nb = nseq * (L // bs + 1) + 4
        kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(nb - 4, dtype=torch.int32, device="cuda").view(nseq, -1)
        q = torch.randn(nseq * L, Hq, D, device="cuda", dtype=torch.bfloat16)
        cu = torch.arange(0, nseq * L + 1, L, dtype=torch.int32, device="cuda")
        ctx = torch.full((nseq,), L, dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        for v in (92, 91):
            ops.PREFILL_WAVES = v
            work = torch.tensor(ops.prefill_work_list([L] * nseq, [L] * nseq, Hq, Hkv), dtype=torch.int32,
                                device="cuda")
            for _ in range(4):
                ops.prefill_attention(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), out, work=work)
            torch.cuda.synchronize()
        print(f"L{L}x{nseq} done", flush=True)
    ops.PREFILL_WAVES = 91


if __name__ == "__main__":
    main()
