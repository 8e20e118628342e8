#!/usr/bin/env python3
"""Single-GPU capacity of the two disaggregated roles (bench.py N > 1).

* prefill role: a prefill-only engine (remote-decode requests, max_tokens=1,
  the KV is released right after "transfer") -> prompts/s and prompt tok/s;
* decode role: a decode engine whose requests are all remote-prefilled: the
  prefill is declared done as soon as blocks are allocated (the KV content
  does not change decode cost), so it measures pure decode steps at the given
  concurrency with contexts ISL..ISL+OSL -> output tok/s and ITL.

With P = prompts/s of a prefill GPU, D = output tok/s of a decode GPU (all
prefill remote) and A = aggregated tok/s (bench.py N=1), an xPyD node with
conditional disaggregation is bounded by
    min(x * P * OSL + y * spare_decode_capacity, ...) ;
tools/role_bench.py prints the projection used in profiles/README.md.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def prompt_gen(seed, isl, vocab):
    import numpy as np

    rs = np.random.RandomState(seed)
    lo = min(1000, vocab // 4)
    return lambda: rs.randint(lo, vocab - lo, size=isl).tolist()


def prefill_role(a):
    import torch

    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
    from dynamo_exp_amd.engine.request import SamplingParams

    eng = LLMEngine(EngineConfig(model=a.model, block_size=a.block_size, max_model_len=a.isl + a.osl + 64,
                                 max_num_seqs=32, max_num_batched_tokens=a.budget, use_cuda_graph=False,
                                 device="cuda", gpu_memory_utilization=0.5, quantization=a.quantization,
                                 kv_cache_dtype=a.kv_cache_dtype))
    gen = prompt_gen(1, a.isl, eng.model_cfg.vocab_size)
    done = []
    eng.prefill_done_hook = lambda r: done.append(r.request_id)
    n = [0]

    def top_up():
        while len(eng.scheduler.waiting) * a.isl < 2 * a.budget:
            n[0] += 1
            eng.add_request(f"p{n[0]}", gen(), SamplingParams(max_tokens=1, ignore_eos=True), remote_decode=True)

    def step():
        top_up()
        eng.step()
        while done:
            eng.finish_transfer(done.pop())

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    p0 = eng.runner.timing["prefill_tokens"]
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    toks = eng.runner.timing["prefill_tokens"] - p0
    return {"role": "prefill", "prompt_tok_s": round(toks / dt, 1), "prompts_s": round(toks / dt / a.isl, 2),
            "ms_per_step": round(dt / a.steps * 1e3, 2), "quantization": a.quantization,
            "kv_cache_dtype": a.kv_cache_dtype}


def decode_role(a):
    import torch

    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
    from dynamo_exp_amd.engine.request import SamplingParams

    conc = a.concurrency
    eng = LLMEngine(EngineConfig(model=a.model, block_size=a.block_size, max_model_len=a.isl + a.osl + 64,
                                 max_num_seqs=conc, max_num_batched_tokens=a.budget, device="cuda",
                                 gpu_memory_utilization=0.9, quantization=a.quantization,
                                 kv_cache_dtype=a.kv_cache_dtype))
    gs = [s for s in (1, 2, 4, 8, 16, 32, 64, 96, 128, 160, 192, 224, 256, 320, 384, 512) if s <= conc]
    if conc not in gs:
        gs.append(conc)
    eng.runner.cfg.graph_sizes = tuple(gs)
    eng.warmup()
    gen = prompt_gen(2, a.isl, eng.model_cfg.vocab_size)
    ready = []
    eng.scheduler.on_remote_prefill = lambda r: ready.append(r.request_id)
    st = dict(gen=0, counting=False, n=0)

    def submit(osl):
        st["n"] += 1

        def on_output(req, toks, lps, fin):
            if st["counting"]:
                st["gen"] += len(toks)
            if fin:
                submit(a.osl)
        eng.add_request(f"d{st['n']}", gen(), SamplingParams(max_tokens=osl, min_tokens=osl, ignore_eos=True),
                        on_output=on_output, remote_prefill=True)

    for i in range(conc):  # staggered progress, as bench.py
        submit(max(1, (i + 1) * a.osl // conc))

    def step():
        eng.step()
        while ready:
            eng.finish_remote_prefill(ready.pop(), 1000, 0.0)

    for _ in range(a.osl + a.warmup):
        step()
    torch.cuda.synchronize()
    st["counting"] = True
    e0, r0 = dict(eng.timing), dict(eng.runner.timing)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    host = {k: round((eng.timing[k] - e0[k]) / a.steps * 1e3, 3) for k in ("schedule", "update", "deliver")}
    host.update({k: round((eng.runner.timing[k] - r0[k]) / a.steps * 1e3, 3) for k in ("decode_prep", "decode_gpu")
                 if isinstance(r0.get(k), float)})
    return {"role": "decode", "concurrency": conc, "output_tok_s": round(st["gen"] / dt, 1),
            "ms_per_step": round(dt / a.steps * 1e3, 2), "ms_per_step_breakdown": host}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--role", choices=["prefill", "decode", "both"], default="both")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--isl", type=int, default=3000)
    ap.add_argument("--osl", type=int, default=150)
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--budget", type=int, default=8192)
    ap.add_argument("--block-size", type=int, default=64)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--agg", type=float, default=None, help="bench.py N=1 tok/s for the projection")
    ap.add_argument("--quantization", default=None, choices=[None, "fp8"], help="fp8: w8a8 e4m3fn projections")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"])
    a = ap.parse_args()
    res = []
    if a.role in ("prefill", "both"):
        res.append(prefill_role(a))
        print(json.dumps(res[-1]), flush=True)
    if a.role in ("decode", "both"):
        import gc

        import torch

        gc.collect()
        torch.cuda.empty_cache()
        res.append(decode_role(a))
        print(json.dumps(res[-1]), flush=True)
    if len(res) == 2:
        P, D = res[0]["prompts_s"], res[1]["output_tok_s"]
        # 1P1D: the decode GPU spends a fraction f = P*OSL/D of its time on the
        # remote-prefilled requests' decode; conditional disagg fills the rest
        # with local prefill at the aggregated rate (upper bound)
        f = min(1.0, P * a.osl / D)
        proj = P * a.osl + (1 - f) * (a.agg or 0.0)
        print(json.dumps({"projection_1P1D_tok_s_per_gpu": round(proj / 2, 1), "decode_busy_on_remote": round(f, 3),
                          "prefill_gpu_output_equiv_tok_s": round(P * a.osl, 1)}), flush=True)


if __name__ == "__main__":
    main()
