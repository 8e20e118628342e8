#!/usr/bin/env python3
"""One rank of a TP-sharded model on one MI355X: the
per-rank projection shapes of Llama-3-70B at TP 4 (hidden 8192, 16 q / 2 KV
heads, FFN 7168 per rank, vocab shard 32064) through the engine's own
decode-GEMM tuner (hand-written small-M kernels vs hipBLASLt per graph size)
and the prefill GEMMs at serving token counts.  No collective runs: the model
is built with a TP group of size 4 whose all-reduces are never called.

  python tools/tp_shapes_bench.py --model llama3-70b --tp 4 --out gpurun_out/tp4_shapes.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=4)
    ap.add_argument("--sizes", default="1,8,16,32,64,96,128,192,256")
    ap.add_argument("--prefill-tokens", default="1024,3072,8192")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from dynamo_exp_amd.models.config import get_config
    from dynamo_exp_amd.models.llama import LlamaForCausalLM, TPGroup

    mc = get_config(a.model)
    dev = torch.device("cuda", 0)
    t0 = time.time()
    m = LlamaForCausalLM(mc, device=dev, tp=TPGroup(None, 0, a.tp)).random_init(0)
    shapes = {n: list(m.layers[0][n].shape) for n in m.LINEARS if n in m.layers[0]}
    shapes["lm_head"] = list(m.lm_head.shape)
    print(f"[tp_shapes] {a.model} tp{a.tp} rank-0 shard built in {time.time() - t0:.1f}s: {shapes}", file=sys.stderr,
          flush=True)
    raw = m.tune_gemms([int(s) for s in a.sizes.split(",")])
    by_nk = {tuple(v): n for n, v in shapes.items()}
    rep = [{"M": r["key"][0], "proj": by_nk.get(tuple(r["key"][1:]), str(r["key"][1:])), "lib_us": r["lib_us"],
            "best_us": r["best_us"], "adopted": r["adopted"],
            "kernel": ("dstream" if r["cfg"] and r["cfg"][0] == __import__("dynamo_exp_amd.ops", fromlist=["x"]).DSTREAM
                       else "skinny") if r["adopted"] else "hipblaslt"} for r in raw]
    out = {"model": a.model, "tp": a.tp, "shapes_NK": shapes, "decode": rep}

    def timed(fn, reps=5):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    pre = []
    for T in (int(v) for v in a.prefill_tokens.split(",")):
        for n, (N, K) in shapes.items():
            x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
            w = m.layers[1][n] if n != "lm_head" else m.lm_head
            us = timed(lambda: torch.matmul(x, w.t()))
            pre.append({"M": T, "proj": n, "us": round(us, 1), "TFLOPs": round(2 * T * N * K / us / 1e6, 1)})
    out["prefill"] = pre
    adopted = {}
    for r in rep:
        adopted[r.get("kernel", "?")] = adopted.get(r.get("kernel", "?"), 0) + 1
    out["adopted_kernels"] = adopted
    # decode GEMM time per step (sum of projections x layers + lm_head) per graph size
    per_step = {}
    for r in rep:
        k = r["M"]
        mult = 1 if r["proj"] == "lm_head" else mc.num_hidden_layers
        per_step[k] = per_step.get(k, 0.0) + mult * min(r["lib_us"], r["best_us"] if r["adopted"] else r["lib_us"])
    out["decode_gemm_ms_per_step"] = {k: round(v / 1e3, 3) for k, v in sorted(per_step.items())}
    print(json.dumps(out["decode_gemm_ms_per_step"]), flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
