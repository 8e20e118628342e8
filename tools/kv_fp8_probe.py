"""FP8 vs bf16 KV cache at serving shapes: decode attention HBM time (B 64-256
streams at ~3100 context) and the prefill path's per-layer dequant pre-pass.

  python -m tools.kv_fp8_probe
"""
import math

import torch

from dynamo_exp_amd import ops
from tools.microbench import bench

FP8 = torch.float8_e4m3fn


def main():
    Hq, Hkv, D, bs = 32, 8, 128, 64
    for B, L in ((64, 3100), (128, 3100), (256, 3100)):
        nbps = L // bs + 1
        nb = B * nbps
        kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        k8, v8 = kc.to(FP8), vc.to(FP8)
        bt = torch.randperm(nb, device="cuda").to(torch.int32).view(B, nbps)
        q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
        ctx = torch.randint(L - 150, L, (B,), dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        mp = ops.decode_num_parts(B, Hkv, L)
        ws = ops.decode_workspace(B, Hq, D, mp, "cuda")
        tb = bench(lambda: ops.decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out, mp, workspace=ws), 30)
        t8 = bench(lambda: ops.decode_attention(q, k8, v8, bt, ctx, 1 / math.sqrt(D), out, mp, workspace=ws), 30)
        tok = int(ctx.sum())
        print(f"decode B{B} L{L}: bf16 {tb:.1f} us ({tok * Hkv * D * 4 / tb / 1e6:.2f} TB/s)  "
              f"fp8 {t8:.1f} us ({tok * Hkv * D * 2 / t8 / 1e6:.2f} TB/s)  speedup {tb / t8:.2f}x", flush=True)
        del kc, vc, k8, v8
    # prefill: 2 prompts x 2800 new tokens (a mixed step's prompt share), per layer
    nseq, Lp = 2, 2800
    nb = nseq * (Lp // bs + 1) + 4
    kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    k8, v8 = kc.to(FP8), vc.to(FP8)
    bt = torch.arange(nb - 4, dtype=torch.int32, device="cuda").view(nseq, -1)
    qp = torch.randn(nseq * Lp, Hq, D, device="cuda", dtype=torch.bfloat16)
    cu = torch.arange(0, nseq * Lp + 1, Lp, dtype=torch.int32, device="cuda")
    ctxp = torch.full((nseq,), Lp, dtype=torch.int32, device="cuda")
    work = torch.tensor(ops.prefill_work_list([Lp] * nseq, [Lp] * nseq, Hq, Hkv), dtype=torch.int32, device="cuda")
    op = torch.empty_like(qp)
    tb = bench(lambda: ops.prefill_attention(qp, kc, vc, bt, cu, ctxp, 1 / math.sqrt(D), op, work=work), 10)
    t8 = bench(lambda: ops.prefill_attention(qp, k8, v8, bt, cu, ctxp, 1 / math.sqrt(D), op, work=work), 10)
    td = bench(lambda: ops.kv_dequant_scratch(k8, v8, bt, ctxp), 20)
    print(f"prefill 2x2800: bf16 {tb:.1f} us, fp8 (dequant + bf16 kernel) {t8:.1f} us, dequant alone {td:.1f} us",
          flush=True)


if __name__ == "__main__":
    main()
