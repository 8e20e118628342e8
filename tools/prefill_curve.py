#!/usr/bin/env python3
"""Prefill-engine TTFT vs ISL on one MI355X (VERDICT r3 next #5b; the
reference derives `max-local-prefill-length` from this curve,
docs/guides/disagg_perf_tuning.md:60-70: "the smallest batch size that
saturates the GPU ... set max-local-prefill-length to the saturation point").

A prefill engine configured as the disaggregated bench's prefill ranks
(whole-prompt steps, 16384-token budget, no prefix hits: every prompt is
fresh random tokens).  Per ISL:

* batch 1: one request alone, TTFT = its prefill step (median of reps),
  prompt tok/s = ISL / TTFT;
* saturating: a queue of prompts worth >= 4 full steps, prompt tok/s over the
  whole drain, TTFT mean / p50 (queueing included).

The saturation point is the smallest ISL whose batch-1 prompt rate reaches
`--frac` (0.9) of the best batch-1 rate (the knee of prefill time per
token): shorter prompts leave a batch-1 prefill engine under-used, so they
are better prefilled locally by the decode engine (conditional
disaggregation).

    python tools/prefill_curve.py --out profiles/r4_prefill_curve.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--isl", default="100,250,500,750,1000,1500,2000,3000,4000,6000,8000,12000,16000")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--budget", type=int, default=16384)
    ap.add_argument("--frac", type=float, default=0.9)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch

    from dynamo_exp_amd.bench.serving import PromptGen
    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
    from dynamo_exp_amd.engine.request import SamplingParams

    from dynamo_exp_amd.models.config import get_config

    max_pos = get_config(a.model).max_position_embeddings
    isls = [int(x) for x in a.isl.split(",") if int(x) + 64 <= max_pos]  # the model's context limit
    cfg = EngineConfig(model=a.model, device=a.device, block_size=64, max_model_len=max(isls) + 64, max_num_seqs=64,
                       max_num_batched_tokens=max(a.budget, max(isls)), chunked_prefill=False,
                       use_cuda_graph=False, gpu_memory_utilization=0.5, seed=1)
    eng = LLMEngine(cfg)
    eng.warmup()
    cuda = torch.device(a.device).type == "cuda"
    sync = (lambda: torch.cuda.synchronize()) if cuda else (lambda: None)
    params = SamplingParams(max_tokens=1, ignore_eos=True)

    def run(prompts):
        first = {}
        t0 = time.perf_counter()
        for i, p in enumerate(prompts):
            eng.add_request(f"q{i}", p, params,
                            on_output=lambda r, t, lp, fin: first.setdefault(r.request_id, time.perf_counter()))
        while eng.has_unfinished():
            eng.step()
        sync()
        t1 = time.perf_counter()
        eng.kv.reset_prefix_cache()
        return t1 - t0, [first[f"q{i}"] - t0 for i in range(len(prompts))]

    rows = []
    for isl in isls:
        gen = PromptGen(isl, isl, eng.model_cfg.vocab_size)
        run([gen()])  # warm this shape
        b1 = [run([gen()])[0] for _ in range(a.reps)]
        t1 = statistics.median(b1)
        n = max(8, -(-4 * a.budget // isl))
        wall, ttfts = run([gen() for _ in range(n)])
        row = {"isl": isl, "batch1_ttft_ms": round(t1 * 1e3, 2), "batch1_tok_s": round(isl / t1),
               "batch1_ms_per_1k_tok": round(t1 * 1e6 / isl, 3),
               "saturated_requests": n, "saturated_tok_s": round(n * isl / wall),
               "saturated_ttft_mean_ms": round(1e3 * sum(ttfts) / n, 1),
               "saturated_ttft_p50_ms": round(1e3 * sorted(ttfts)[n // 2], 1)}
        print(json.dumps(row), flush=True)
        rows.append(row)
    best = max(r["saturated_tok_s"] for r in rows)
    best1 = max(r["batch1_tok_s"] for r in rows)
    # the knee: the smallest ISL whose batch-1 rate reaches frac of the best batch-1 rate
    sat = next((r["isl"] for r in rows if r["batch1_tok_s"] >= a.frac * best1), None)
    out = {"model": a.model, "engine": "prefill role: whole-prompt steps, budget %d tokens, fresh prompts" % a.budget,
           "dtype": "bf16", "data": "synthetic random-token prompts, random-init weights",
           "best_saturated_tok_s": best, "best_batch1_tok_s": best1, "saturation_fraction": a.frac,
           "saturation_isl": sat, "rows": rows}
    print(json.dumps({k: out[k] for k in ("best_saturated_tok_s", "saturation_isl")}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
