"""Which decode-size GEMM kernel the warm-up tuner adopts per (batch size,
projection) for Llama-3-8B (random weights): hipBLASLt, the register-fed
skinny kernel, or the deep-stream kernel (ds).  Prints one JSON line per key and a per-kernel count.
(The w8a8 model has no hand-kernel candidates since round 6: its decode GEMMs are hipBLASLt's fp8 kernels.)

  python -m tools.tune_report [--model llama3-70b] [--out profiles/...]
"""
import argparse
import collections
import json
import sys

import torch

sys.path.insert(0, ".")
from dynamo_exp_amd import ops  # noqa: E402
from dynamo_exp_amd.models.config import get_config  # noqa: E402
from dynamo_exp_amd.models.llama import LlamaForCausalLM  # noqa: E402


def kind(cfg) -> str:
    if cfg is None:
        return "hipblaslt"
    if cfg[0] == ops.DSTREAM:
        return "dstream"
    return "skinny"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--sizes", default="1,2,4,8,16,24,32,48,64,80,96,112,128,160,192,224,256")
    ap.add_argument("--model", default="llama3-8b")
    a = ap.parse_args()
    m = LlamaForCausalLM(get_config(a.model), device=torch.device("cuda:0")).random_init(1)
    names = {}
    L0 = m.layers[0]
    for n in m.LINEARS:
        names[tuple(L0[n].shape)] = n
    names[tuple(m.lm_head.shape)] = "lm_head"
    plan = m.gemm_plan
    rows = []
    for M in [int(s) for s in a.sizes.split(",")]:
        for r in m.tune_gemms([M]):
            N, K = r["key"][1], r["key"][2]
            row = {"M": M, "proj": names.get((N, K), f"{N}x{K}"), "lib_us": r["lib_us"], "best_us": r["best_us"],
                   "best": kind(r["cfg"]) if r["cfg"] is not None else None, "adopted": r["adopted"],
                   "kernel": kind(plan.get(r["key"])), "cfg": r["cfg"]}
            rows.append(row)
            print(json.dumps(row), flush=True)
    cnt = collections.Counter(r["kernel"] for r in rows)
    print(json.dumps({"adopted_kernels": dict(cnt)}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"model": a.model, "rows": rows, "adopted_kernels": dict(cnt)}, f, indent=1)


if __name__ == "__main__":
    main()
