#!/usr/bin/env python3
"""Headline benchmark: Llama-3-8B serving throughput on MI355X.

Metric (BASELINE.json): output tokens/sec of the node + p50 TTFT, Llama-3-8B,
synthetic ISL 3000 / OSL 150 requests with ignore_eos (the reference's
genai-perf methodology, examples/llm/benchmarks/perf.sh:17-54), closed loop at
a fixed per-GPU concurrency (weak scaling: per-GPU load fixed as N grows).

* N = 1: aggregated engine (prefill + decode on one GPU, TP1, bf16).
* N > 1 (torchrun, one rank per GPU): disaggregated xPyD with x = y = N/2
  (1P1D .. 4P4D).  Each decode rank owns its requests; prompts longer than the
  conditional-disagg threshold are prefilled on its paired prefill rank and the
  KV blocks are shipped back over RCCL (xGMI) send/recv; decode ranks prefill
  locally when the prefill queue is full (conditional disaggregation,
  examples/llm/components/disagg_router.py:24-66).

A "step" is one engine iteration on each rank; W untimed warmup steps, then
exactly K timed steps bracketed by barrier + synchronize; value = total output
tokens generated inside the window over all ranks / max elapsed over ranks.
Weights are random-init with the real architecture; data is synthetic.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "output tokens/sec (node) + p50 TTFT at fixed QPS, Llama-3-8B disagg 1P+1D..4P+4D"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--isl", type=int, default=3000)
    ap.add_argument("--osl", type=int, default=150)
    ap.add_argument("--concurrency", type=int, default=128,
                    help="in-flight requests per GPU (decode ranks own concurrency*N/n_decode each)")
    ap.add_argument("--block-size", type=int, default=64)
    ap.add_argument("--max-batched-tokens", type=int, default=None,
                    help="per-step token budget (default 8192 chunked, 16384 prefill-first)")
    ap.add_argument("--policy", default="chunked", choices=["chunked", "prefill-first"],
                    help="chunked = mixed prefill-chunk + decode batches; prefill-first = whole-prompt prefill steps")
    ap.add_argument("--max-prefill-streak", type=int, default=2)
    ap.add_argument("--min-prefill-tokens", type=int, default=8000,
                    help="prefill batching: while streams decode, hold new prompts until this many tokens are "
                         "queued ... (0 = off; profiles/r1_prefill_batching_sweep.json)")
    ap.add_argument("--max-prefill-delay", type=float, default=0.3, help="... or the oldest waited this long (s)")
    ap.add_argument("--max-local-prefill", type=int, default=1000,
                    help="conditional disagg: prompts longer than this go to the prefill rank")
    ap.add_argument("--max-prefill-queue", type=int, default=None,
                    help="conditional disagg: remote only while the shared prefill queue is shorter than this "
                         "(default 4 per prefill rank: a prefill step pulls ~3 ISL-3000 prompts, so each rank "
                         "stays fed while the queueing delay stays ~4 prompts' worth of one rank's time)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--gemm-report", default=None, help="write the decode-GEMM tuning table (JSON) here")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--cpu", action="store_true", help="CPU reference path (tests only)")
    ap.add_argument("--quantization", default=None, choices=[None, "fp8"],
                    help="fp8 = w8a8 e4m3fn projections (reported as dtype fp8; the headline is bf16)")
    ap.add_argument("--num-gpu-blocks", type=int, default=None)
    ap.add_argument("--gpu-mem-util", type=float, default=None)
    ap.add_argument("--p2p-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = host-staged KV transfer (lets >1 rank share one GPU for functional tests)")
    a = ap.parse_args()
    if a.max_batched_tokens is None:
        a.max_batched_tokens = 8192 if a.policy == "chunked" else 16384
    return a


def stagger_lengths(n: int, osl: int) -> list[int]:
    """Output lengths of the initial streams: i * osl / n for i = 1..n (the
    last one is a full-length request), i.e. progress spread uniformly."""
    return [max(1, (i + 1) * osl // n) for i in range(n)]


class PromptGen:
    """Distinct random-token prompts (no accidental prefix sharing), numpy-fast
    so the load generator stays off the engine's critical path."""

    def __init__(self, seed: int, n: int, vocab: int):
        import numpy as np

        self.rs = np.random.RandomState(seed)
        self.n, self.vocab = n, vocab

    def __call__(self) -> list[int]:
        lo = min(1000, self.vocab // 4)
        return self.rs.randint(lo, self.vocab - lo, size=self.n).tolist()


def run_aggregated(args, dev):
    import torch

    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
    from dynamo_exp_amd.engine.request import SamplingParams

    cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=args.isl + args.osl + 64,
                       max_num_seqs=max(args.concurrency, 1), max_num_batched_tokens=args.max_batched_tokens,
                       max_prefill_streak=args.max_prefill_streak, use_cuda_graph=not args.no_graph,
                       chunked_prefill=args.policy == "chunked", device=str(dev), seed=args.seed,
                       quantization=args.quantization, min_prefill_tokens=args.min_prefill_tokens,
                       max_prefill_delay=args.max_prefill_delay)
    t0 = time.time()
    eng = LLMEngine(cfg)
    gs = [s for s in (1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256) if s <= args.concurrency]
    if args.concurrency not in gs:
        gs.append(args.concurrency)
    eng.runner.cfg.graph_sizes = tuple(gs)
    cap = eng.warmup()
    if args.gemm_report:
        with open(args.gemm_report, "w") as f:
            json.dump(eng.gemm_report, f, indent=1)
    log(args, f"engine ready in {time.time() - t0:.1f}s (graphs {cap:.1f}s), kv blocks {eng.runner.num_blocks}")
    gen_prompt = PromptGen(args.seed, args.isl, eng.model_cfg.vocab_size)
    state = dict(gen=0, ttft=[], itl=[], counting=False, n=0)

    def submit(osl=None):
        state["n"] += 1
        rid = f"r{state['n']}"
        osl = osl or args.osl
        params = SamplingParams(temperature=0.0, max_tokens=osl, min_tokens=osl, ignore_eos=True)
        arrival = time.perf_counter()
        last = [None]

        def on_output(req, toks, lps, fin, arrival=arrival, last=last):
            now = time.perf_counter()
            if state["counting"]:
                state["gen"] += len(toks)
                if req.first_token_time is not None and len(req.output) == len(toks) and toks:
                    state["ttft"].append(req.first_token_time - arrival)
                elif last[0] is not None and toks:
                    state["itl"].append((now - last[0]) / len(toks))
            last[0] = now
            if fin:
                if osl != args.osl:
                    state["fill"] -= 1
                submit()

        eng.add_request(rid, gen_prompt(), params, on_output=on_output)

    # steady-state fill (before the W warmup steps): the initial streams get
    # staggered output lengths so their completions -- and the full ISL/OSL
    # requests that replace them -- are spread uniformly over an OSL cycle;
    # without it every stream starts and ends in lock-step and short K/W
    # windows would measure the start-up transient instead of serving.
    fill = stagger_lengths(args.concurrency, args.osl)
    state["fill"] = sum(1 for o in fill if o != args.osl)
    for o in fill:
        submit(o)
    t_fill = time.perf_counter()
    fill_steps = 0
    while state["fill"] > 0:
        eng.step()
        fill_steps += 1
    log(args, f"steady-state fill: {fill_steps} steps in {time.perf_counter() - t_fill:.1f}s")
    for _ in range(args.warmup):
        eng.step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    state["counting"] = True
    s0 = dict(eng.stats)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        eng.step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    s1 = eng.stats
    itl = sorted(state["itl"])
    extra = dict(prefill_steps=s1["prefill_steps"] - s0["prefill_steps"],
                 decode_steps=s1["decode_steps"] - s0["decode_steps"],
                 mixed_steps=s1["mixed_steps"] - s0["mixed_steps"],
                 itl_p50_ms=round(itl[len(itl) // 2] * 1000, 2) if itl else None)
    log(args, "engine timing (s, incl. warmup): " + str({k: round(v, 3) for k, v in eng.timing.items()}) +
        " runner: " + str({k: round(v, 3) if isinstance(v, float) else v for k, v in eng.runner.timing.items()}))
    return state["gen"], elapsed, state["ttft"], extra


def log(args, msg):
    if args.verbose or os.environ.get("RANK", "0") == "0":
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # watchdog: a wedged multi-rank run dumps every thread's stack and exits
    # instead of holding the node (default 25 min for N > 1)
    dump_after = os.environ.get("DX_DUMP_AFTER") or ("1500" if world > 1 else None)
    if dump_after:
        import faulthandler

        faulthandler.dump_traceback_later(float(dump_after), exit=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    if args.cpu:
        dev = torch.device("cpu")
    else:
        local = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        from dynamo_exp_amd.disagg.bench_disagg import run_disaggregated

        gen, elapsed, ttft, extra = run_disaggregated(args, dev, rank, world)
        parallelism = f"disagg-{world // 2}P{world - world // 2}D-tp1"
    else:
        gen, elapsed, ttft, extra = run_aggregated(args, dev)
        parallelism = "agg-tp1"
    if rank == 0:
        ttft = sorted(ttft)
        p50 = ttft[len(ttft) // 2] * 1000 if ttft else None
        p99 = ttft[min(len(ttft) - 1, int(len(ttft) * 0.99))] * 1000 if ttft else None
        value = gen / elapsed if elapsed > 0 else 0.0
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(1, args.steps) * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp8-w8a8" if args.quantization == "fp8" else "bf16",
            "data": "synthetic (random-token prompts, random-init weights of the real architecture)",
            "ttft_p50_ms": None if p50 is None else round(p50, 2),
            "ttft_p99_ms": None if p99 is None else round(p99, 2),
            "output_tokens": gen,
            "elapsed_s": round(elapsed, 3),
            "config": {
                "model": "Llama-3-8B" if args.model == "llama3-8b" else args.model,
                "global_batch": args.concurrency * world,
                "seq_len": args.isl + args.osl,
                "isl": args.isl,
                "osl": args.osl,
                "concurrency_per_gpu": args.concurrency,
                "policy": args.policy,
                "max_batched_tokens": args.max_batched_tokens,
                "prefill_batching": [args.min_prefill_tokens, args.max_prefill_delay],
                "parallelism": parallelism,
                **extra,
            },
        }
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
