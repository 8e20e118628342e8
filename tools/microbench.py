"""Kernel microbenchmarks on the GPU (wall time via HIP events, interleaved
repetitions): Llama-3-8B GEMM shapes through hipBLASLt, and the HIP kernels
(prefill / decode attention, rmsnorm, rope, silu) at serving shapes."""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamo_exp_amd import ops  # noqa: E402


def bench(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def gemms(M):
    out = {}
    H, F = 4096, 14336
    for name, (K, N) in {"qkv": (H, 6144), "o": (H, H), "gate_up": (H, 2 * F), "down": (F, H),
                         "lm_head": (H, 128256)}.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        us = bench(lambda: torch.matmul(x, w.t()))
        out[f"gemm_{name}_M{M}"] = {"us": round(us, 1), "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}
    return out


def attention(Hq: int = 32, Hkv: int = 8):
    """Prefill / decode attention at (Hq, Hkv) heads: 32 / 8 = Llama-3-8B;
    16 / 2 = one rank of Llama-3-70B at TP 4 (config 4); 64 / 8 = 70B at TP 1."""
    res = {}
    D, bs = 128, int(os.environ.get("DX_MB_BLOCK", "64"))
    for L, nseq in (() if os.environ.get("DX_MB_DECODE_ONLY") else ((3000, 5), (8000, 2), (16000, 1))):
        nb = nseq * (L // bs + 1) + 4
        kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(nb - 4, dtype=torch.int32, device="cuda").view(nseq, -1)
        q = torch.randn(nseq * L, Hq, D, device="cuda", dtype=torch.bfloat16)
        cu = torch.arange(0, nseq * L + 1, L, dtype=torch.int32, device="cuda")
        ctx = torch.full((nseq,), L, dtype=torch.int32, device="cuda")
        work = torch.tensor(ops.prefill_work_list([L] * nseq, [L] * nseq, Hq, Hkv), dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        us = bench(lambda: ops.prefill_attention(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), out, work=work), 10)
        flops = nseq * 4 * (L * L / 2) * D * Hq
        res[f"prefill_attn_L{L}x{nseq}"] = {"us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 1)}
    # engine-shaped prefill batches (DX_MB_PREFILL_MIX=1): an 8064-token mixed step's prompt pieces as
    # (new tokens, context) -- a prompt's tail behind its cached head, whole prompts, a prompt's head
    mixes = {"mixA": ((2064, 3000), (3000, 3000), (3000, 3000)),
             "mixB": ((1032, 3000), (3000, 3000), (3000, 3000), (1032, 1032)),
             "mixC": ((3000, 3000), (3000, 3000), (2064, 2064)),
             "mixD": ((4032, 3000 + 1032), (4032, 4032))}
    for name, cases in (mixes.items() if os.environ.get("DX_MB_PREFILL_MIX") else ()):
        nseq = len(cases)
        nbps = max(c for _, c in cases) // bs + 1
        kc = torch.randn(nseq * nbps + 4, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(nseq * nbps, dtype=torch.int32, device="cuda").view(nseq, nbps)
        qlens = [qn for qn, _ in cases]
        ctxs = [c for _, c in cases]
        T = sum(qlens)
        q = torch.randn(T, Hq, D, device="cuda", dtype=torch.bfloat16)
        cu = torch.tensor([0] + torch.tensor(qlens).cumsum(0).tolist(), dtype=torch.int32, device="cuda")
        ctx = torch.tensor(ctxs, dtype=torch.int32, device="cuda")
        work = torch.tensor(ops.prefill_work_list(qlens, ctxs, Hq, Hkv), dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        us = bench(lambda: ops.prefill_attention(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), out, work=work), 10)
        flops = sum(4 * D * Hq * (qn * (c - qn) + qn * (qn + 1) / 2) for qn, c in cases)
        res[f"prefill_attn_{name}"] = {"us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 1), "cases": cases}
    shapes = ((64, 3100), (128, 3100), (256, 3100), (8, 16000))
    if os.environ.get("DX_MB_DECODE_ONLY"):  # the partition sweep: low-batch and long-context points too
        shapes += ((1, 3100), (16, 3100), (32, 3100), (32, 8000), (2, 16000))
    for B, L in shapes:
        nbps = L // bs + 1
        nb = B * nbps
        kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        if os.environ.get("DX_MB_KV_FP8"):  # e4m3fn cache (scales 1): half the bytes per token
            kc, vc = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
        bt = torch.randperm(nb, device="cuda").to(torch.int32).view(B, nbps)
        q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
        ctx = torch.full((B,), L, dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        mp = ops.decode_num_parts(B, Hkv, L)
        ws = ops.decode_workspace(B, Hq, D, mp, "cuda")
        us = bench(lambda: ops.decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out, mp, workspace=ws))
        byts = B * L * Hkv * D * 2 * kc.element_size()
        res[f"decode_attn_B{B}_L{L}"] = {"us": round(us, 1), "TB/s": round(byts / us / 1e6, 2), "parts": mp}
    return res


def decode_only():
    """Decode attention at serving shapes + checksum vs the default kernel's output."""
    res = {}
    Hq, Hkv, D, bs = 32, 8, 128, 64
    torch.manual_seed(0)
    for B, L in ((128, 3100), (256, 3100), (32, 8000)):
        nbps = L // bs + 1
        nb = B * nbps
        kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        if os.environ.get("DX_MB_KV_FP8"):  # e4m3fn cache (scales 1): half the bytes per token
            kc, vc = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
        bt = torch.randperm(nb, device="cuda").to(torch.int32).view(B, nbps)
        q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
        ctx = torch.randint(L - 200, L, (B,), dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        mp = ops.decode_num_parts(B, Hkv, L)
        ws = ops.decode_workspace(B, Hq, D, mp, "cuda")
        us = bench(lambda: ops.decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out, mp, workspace=ws), 30)
        byts = int(ctx.sum().item()) * Hkv * D * 2 * 2
        # fp32 reference on 4 sequences
        from dynamo_exp_amd.ops import reference as R
        cu = torch.arange(5, dtype=torch.int32, device="cuda")
        ref = R.paged_attention(q[:4].float(), kc, vc, bt[:4], cu, ctx[:4], 1 / math.sqrt(D), bs)
        err = float((out[:4].float() - ref.float()).abs().max())
        res[f"decode_attn_B{B}_L{L}"] = {"us": round(us, 1), "TB/s": round(byts / us / 1e6, 2), "max_err": err}
    return res


def elementwise():
    res = {}
    for T in (128, 16384):
        x = torch.randn(T, 4096, device="cuda", dtype=torch.bfloat16)
        r = torch.randn_like(x)
        w = torch.ones(4096, device="cuda", dtype=torch.bfloat16)
        us = bench(lambda: ops.add_rmsnorm(x, r, w, 1e-5, out=x))
        res[f"add_rmsnorm_T{T}"] = {"us": round(us, 1), "TB/s": round(T * 4096 * 2 * 3 / us / 1e6, 2)}
        gu = torch.randn(T, 2 * 14336, device="cuda", dtype=torch.bfloat16)
        o = torch.empty(T, 14336, device="cuda", dtype=torch.bfloat16)
        us = bench(lambda: ops.silu_and_mul(gu, out=o))
        res[f"silu_mul_T{T}"] = {"us": round(us, 1), "TB/s": round(T * 14336 * 2 * 3 / us / 1e6, 2)}
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="all")
    ap.add_argument("--heads", default="32,8", help="q heads,kv heads of the attention benchmarks")
    a = ap.parse_args()
    hq, hkv = (int(v) for v in a.heads.split(","))
    res = {}
    if a.what in ("all", "gemm"):
        for M in (128, 16384):
            res.update(gemms(M))
    if a.what in ("all", "attn"):
        res.update(attention(hq, hkv))
    if a.what == "decode":
        res.update(decode_only())
    if a.what in ("all", "elem"):
        res.update(elementwise())
    print(json.dumps(res, indent=1))
