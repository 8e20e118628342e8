"""Multi-turn prefix-reuse benchmark for the pinned-host KV tier.

Reference experiment (BASELINE.md row "KV host offload vs GPU-only prefix
caching": 10 multi-turn rounds, 80 users, TTFT per round; docs/architecture.md:91,
docs/images/kv_manager.png).  Each user holds a conversation: round 0 sends a
`--first`-token prompt, every later round resends the whole history (previous
prompt + the previous answer) plus a `--turn`-token follow-up.  All users send
round r together; TTFT is measured per request in the engine (arrival ->
first token, engine clock).  The device KV pool is sized (`--gpu-blocks`) below
the users' total history so prefixes get evicted between rounds; with
`--host-blocks` > 0 evicted blocks are demoted to pinned host memory and
promoted back on a later hit instead of being recomputed.

    python tools/multiturn_bench.py --model deepseek-r1-distill-llama-8b --users 32 --rounds 6 \
        --gpu-blocks 700 --host-blocks 0,2400 --out multiturn.json

Prints one JSON line per host-tier setting: per-round TTFT p50 / mean and
prefix-hit tokens (device, host).  Synthetic prompts, random-init weights.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(a, host_blocks: int) -> dict:
    import numpy as np
    import torch

    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
    from dynamo_exp_amd.engine.request import SamplingParams

    dev = "cpu" if a.cpu else "cuda:0"
    cfg = EngineConfig(model=a.model, block_size=a.block_size, num_gpu_blocks=a.gpu_blocks,
                       max_model_len=a.first + a.rounds * (a.turn + a.osl) + 64, max_num_seqs=a.users,
                       max_num_batched_tokens=a.max_batched_tokens, device=dev, host_kv_blocks=host_blocks,
                       use_cuda_graph=not a.cpu, seed=a.seed)
    eng = LLMEngine(cfg)
    if not a.cpu:
        eng.warmup()
    vocab = eng.model_cfg.vocab_size
    rs = np.random.RandomState(a.seed)
    lo = min(1000, vocab // 4)

    def toks(n):
        return rs.randint(lo, vocab - lo, size=n).tolist()

    hist = [toks(a.first) for _ in range(a.users)]
    rounds = []
    km = eng.kv
    for r in range(a.rounds):
        if r > 0:
            hist = [h + toks(a.turn) for h in hist]
        ttft, outs = {}, {}
        arrival = {}
        host_hit0 = km.host_hit_tokens
        hits = []

        def on_output(req, new, lps, fin, i=None):
            if req.first_token_time is not None and i not in ttft:
                ttft[i] = req.first_token_time - arrival[i]
            if fin:
                outs[i] = list(req.output)
                hits.append(req.num_prefix_hit)

        t0 = time.perf_counter()
        for i, h in enumerate(hist):
            arrival[i] = time.perf_counter()
            eng.add_request(f"u{i}r{r}", list(h), SamplingParams(max_tokens=a.osl, min_tokens=a.osl, ignore_eos=True),
                            on_output=lambda req, n, l, f, i=i: on_output(req, n, l, f, i))
        while len(outs) < a.users:
            eng.step()
        if not a.cpu:
            torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        hist = [hist[i] + outs[i] for i in range(a.users)]
        xs = sorted(ttft.values())
        host_hit = km.host_hit_tokens - host_hit0
        rounds.append({"round": r, "prompt_tokens": sum(len(h) for h in hist) - sum(len(o) for o in outs.values()),
                       "ttft_p50_ms": round(xs[len(xs) // 2] * 1000, 2), "ttft_mean_ms": round(sum(xs) / len(xs) * 1000, 2),
                       "prefix_hit_tokens": int(sum(hits)), "host_hit_tokens": int(host_hit),
                       "wall_s": round(wall, 3)})
        print(f"[multiturn host={host_blocks}] {json.dumps(rounds[-1])}", file=sys.stderr, flush=True)
    res = {"host_blocks": host_blocks, "gpu_blocks": eng.runner.num_blocks, "rounds": rounds,
           "ttft_mean_ms_rounds_1plus": round(sum(x["ttft_mean_ms"] for x in rounds[1:]) / max(1, len(rounds) - 1), 2),
           "host_tier": dict(eng.kv.host.stats) if eng.kv.host is not None else None}
    del eng
    if not a.cpu:
        torch.cuda.empty_cache()
    return res


def main(argv=None):
    ap = argparse.ArgumentParser(prog="multiturn_bench")
    ap.add_argument("--model", default="deepseek-r1-distill-llama-8b")
    ap.add_argument("--users", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--first", type=int, default=2000)
    ap.add_argument("--turn", type=int, default=100)
    ap.add_argument("--osl", type=int, default=150)
    ap.add_argument("--block-size", type=int, default=64)
    ap.add_argument("--gpu-blocks", type=int, default=700)
    ap.add_argument("--host-blocks", default="0,2400", help="comma list; 0 = GPU-only prefix caching")
    ap.add_argument("--max-batched-tokens", type=int, default=8192)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    results = [run(a, int(h)) for h in a.host_blocks.split(",")]
    for r in results:
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"model": a.model, "users": a.users, "rounds": a.rounds, "first": a.first, "turn": a.turn,
                       "osl": a.osl, "data": "synthetic prompts, random-init weights", "runs": results}, f, indent=1)
    return results


if __name__ == "__main__":
    main()
