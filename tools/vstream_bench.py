"""Decode-size projection GEMMs at the Llama-3-8B shapes: hipBLASLt vs the
register-streamed kernel (csrc/kernels/vstream_gemm.hip, every config) vs the
best of the older small-M kernels (skinny_gemm / wstream_gemm), weights cold
(rotating over 32 copies > the 256 MB Infinity Cache, as in a decode step).
Every vstream config is checked against fp32 before it is timed.

  python tools/vstream_bench.py --out gpurun_out/vstream.json [--old]
"""
import argparse
import json

import torch

from dynamo_exp_amd import ops
from tools.skinny_bench import SHAPES, timed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/vstream.json")
    ap.add_argument("--ms", default="64,128,256")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--old", action="store_true", help="also sweep the skinny / wstream configs")
    a = ap.parse_args()
    res = {}
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(a.copies)]
        gb = N * K * 2 / 1e9
        for M in map(int, a.ms.split(",")):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            want = (x.float() @ ws[0].float().t())
            lib = timed(lambda: [torch.matmul(x, w.t()) for w in ws]) / len(ws)
            rows = []
            for cfg in ops.vstream_configs(M, N, K):
                for nt in (0, 1):
                    c = cfg[:6] + (nt,)
                    got = ops.skinny_linear(x, ws[0], c).float()
                    err = ((got - want).abs().max() / want.abs().max()).item()
                    if not err < 2e-2:
                        raise SystemExit(f"vstream {c} {name} M{M}: relative error {err:.3g}")
                    t = timed(lambda: [ops.skinny_linear(x, w, c) for w in ws]) / len(ws)
                    rows.append((t, c))
            rows.sort()
            r = {"lib_us": round(lib, 1), "lib_TBs": round(gb / lib * 1e3, 2),
                 "vs_us": round(rows[0][0], 1), "vs_TBs": round(gb / rows[0][0] * 1e3, 2), "vs_cfg": rows[0][1],
                 "vs_top5": [(round(t, 1), c) for t, c in rows[:5]]}
            if a.old:
                old = []
                for cfg in ops.skinny_configs(M, N, K) + ops.wstream_configs(M, N, K):
                    old.append((timed(lambda: [ops.skinny_linear(x, w, cfg) for w in ws]) / len(ws), cfg))
                old.sort()
                r["old_us"], r["old_cfg"] = round(old[0][0], 1), old[0][1]
            res[f"{name}_M{M}"] = r
            print(name, M, r, flush=True)
        del ws
        torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
