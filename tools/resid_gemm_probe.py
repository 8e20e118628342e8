"""Does folding the residual add into the prefill O / down GEMM pay?

Today (TP 1, prefill-size M on hipBLASLt):  h = x . W^T  (writes h),
then add_rmsnorm reads h and the residual, writes the residual and the normed
rows: four [M, 4096] bf16 passes.  Folded:  residual.addmm_(x, W^T) -- the
library's beta = 1 epilogue reads the residual tile and writes the sum --
then a plain rmsnorm reads the residual and writes the normed rows: two
passes outside the GEMM, one extra read inside it.

Llama-3-8B O (4096 x 4096) and down (4096 x 14336) weights of 32 layers,
rotated past the Infinity Cache; random activations.  Prints us per
(GEMM + norm) pair for both forms, and the GEMM alone at beta 0 / 1.

  python -m tools.resid_gemm_probe [--out profiles/...]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from dynamo_exp_amd import ops  # noqa: E402


def timed(fn, n_layers, iters=3):
    for i in range(n_layers):
        fn(i)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        for i in range(n_layers):
            fn(i)
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) * 1e3 / (iters * n_layers), 2)


@torch.inference_mode()
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--ms", default="3000,5728,8192")
    ap.add_argument("--layers", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    H, F, L = 4096, 14336, a.layers
    Wo = [torch.randn(H, H, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
    Wd = [torch.randn(H, F, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
    nw = torch.rand(H, device=dev, dtype=torch.bfloat16) + 0.5
    rows = []
    for M in [int(m) for m in a.ms.split(",")]:
        for name, Ws, K in (("o", Wo, H), ("down", Wd, F)):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            res0 = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
            res = res0.clone()
            h = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
            xb = torch.empty(M, H, device=dev, dtype=torch.bfloat16)

            def today(i):
                torch.matmul(x, Ws[i].t(), out=h)
                ops.add_rmsnorm(h, res, nw, 1e-5, out=h)

            def folded(i):
                res.addmm_(x, Ws[i].t())
                ops.rmsnorm(res, nw, 1e-5, out=xb)

            def gemm0(i):
                torch.matmul(x, Ws[i].t(), out=h)

            def gemm1(i):
                res.addmm_(x, Ws[i].t())

            r = {"M": M, "proj": name}
            for _ in range(2):  # interleaved rounds, best of
                for k, fn in (("today", today), ("folded", folded), ("gemm_beta0", gemm0), ("gemm_beta1", gemm1)):
                    res.copy_(res0)
                    t = timed(fn, L)
                    r[k] = min(r.get(k, 1e9), t)
            r["gain_us"] = round(r["today"] - r["folded"], 2)
            # numerics of one layer against fp32
            ref32 = res0.float() + x.float() @ Ws[0].float().t()
            res.copy_(res0)
            torch.matmul(x, Ws[0].t(), out=h)
            ops.add_rmsnorm(h, res, nw, 1e-5, out=h)
            e_today = (res.float() - ref32).abs().max().item()
            res.copy_(res0)
            res.addmm_(x, Ws[0].t())
            e_fold = (res.float() - ref32).abs().max().item()
            r["max_err_today"], r["max_err_folded"] = round(e_today, 4), round(e_fold, 4)
            print(json.dumps(r), flush=True)
            rows.append(r)
    if a.out:
        with open(a.out, "w") as f:
            f.write("# tools/resid_gemm_probe.py: us per (GEMM + norm), Llama-3-8B O / down, 32 layers' weights\n")
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
