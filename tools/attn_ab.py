"""A/B of prefill-attention kernel variants selected by ops.PREFILL_WAVES
(csrc/kernels/attn_prefill.hip: 91 = current, 92 = the pre-round-4 loop without
the deferred rescale / matrix-pipe row sum / static priority / widened
epilogue), interleaved on one box at the headline shapes (5 x 3000, 2 x 8000, 1 x 16000).

  python -m tools.attn_ab
"""
import json
import math

import torch

from dynamo_exp_amd import ops
from tools.microbench import bench


def run(variants=(92, 91), rounds=3):
    Hq, Hkv, D, bs = 32, 8, 128, 64
    res = {}
    for L, nseq in ((3000, 5), (8000, 2), (16000, 1)):
        nb = nseq * (L // bs + 1) + 4
        kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(nb - 4, dtype=torch.int32, device="cuda").view(nseq, -1)
        q = torch.randn(nseq * L, Hq, D, device="cuda", dtype=torch.bfloat16)
        cu = torch.arange(0, nseq * L + 1, L, dtype=torch.int32, device="cuda")
        ctx = torch.full((nseq,), L, dtype=torch.int32, device="cuda")
        works = {}
        for v in variants:  # the work items' token count depends on the variant's waves per workgroup
            ops.PREFILL_WAVES = v
            works[v] = torch.tensor(ops.prefill_work_list([L] * nseq, [L] * nseq, Hq, Hkv), dtype=torch.int32,
                                    device="cuda")
        flops = nseq * 4 * (L * L / 2) * D * Hq
        outs = {}
        for v in variants:
            ops.PREFILL_WAVES = v
            o = torch.empty_like(q)
            ops.prefill_attention(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), o, work=works[v])
            outs[v] = o
        ref = outs[variants[0]].float()
        for v in variants[1:]:
            assert (outs[v].float() - ref).abs().max().item() < 2e-2, v
        tf = {v: [] for v in variants}
        for _ in range(rounds):
            for v in variants:
                ops.PREFILL_WAVES = v
                out = outs[v]
                wk = works[v]
                us = bench(lambda: ops.prefill_attention(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), out, work=wk), 10)
                tf[v].append(round(flops / us / 1e6, 1))
        res[f"L{L}x{nseq}"] = {str(v): max(t) for v, t in tf.items()}
        print(f"L{L}x{nseq}", tf, flush=True)
    ops.PREFILL_WAVES = 91
    return res


if __name__ == "__main__":
    print(json.dumps(run(), indent=1))
