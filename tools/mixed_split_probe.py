"""Could a mixed step run its decode rows as a SEPARATE forward on a second
stream, beside the prefill rows' forward?  The two are independent (different
sequences), the decode forward is memory-bound (KV + weight streaming, VALU
dot products in decode attention) and the prefill forward MFMA-bound, so they
might share the GPU better than the one fused forward runs them back to back.

Llama-3-8B, random weights, at the headline's mixed-step shape (2 prompts x
2800 new tokens + 128 decode streams at ~3100 context): per-forward times of
  fused   -- today's mixed forward (decode rows ride in the big GEMMs, decode
             attention serial after the prefill attention),
  prefill -- the prefill rows alone,  decode -- a captured decode step alone,
  serial  -- prefill forward then decode graph,
  split   -- prefill forward on the main stream || decode graph on a side stream.

  python -m tools.mixed_split_probe [--out profiles/...]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from dynamo_exp_amd import ops  # noqa: E402
from dynamo_exp_amd.models.config import get_config  # noqa: E402
from dynamo_exp_amd.models.llama import AttnMeta, LlamaForCausalLM  # noqa: E402


def timed(fn, iters=6, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) / iters, 3)


@torch.inference_mode()
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--prompts", type=int, default=2)
    ap.add_argument("--chunk", type=int, default=2800)
    ap.add_argument("--decode", type=int, default=128)
    ap.add_argument("--ctx", type=int, default=3100)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = get_config("llama3-8b")
    m = LlamaForCausalLM(cfg, device=dev).random_init(1)
    B, P, C, L = a.decode, a.prompts, a.chunk, a.ctx
    m.tune_gemms([B])
    bs = 64
    nq, nkv, D = m.n_q, m.n_kv, m.head_dim
    nb_d, nb_p = -(-(L + 1) // bs), -(-C // bs)
    nblocks = B * nb_d + P * nb_p + 1
    kv = torch.randn(cfg.num_hidden_layers, 2, nblocks, nkv, bs, D, device=dev, dtype=torch.bfloat16).mul_(0.5)
    caches = [(kv[i, 0], kv[i, 1]) for i in range(cfg.num_hidden_layers)]
    # decode rows: sequence b owns blocks 1 + b * nb_d ..; its new token at position L - 1
    dbt = (1 + torch.arange(B * nb_d, device=dev, dtype=torch.int32)).view(B, nb_d)
    dctx = torch.full((B,), L, device=dev, dtype=torch.int32)
    dpos = torch.full((B,), L - 1, device=dev, dtype=torch.int64)
    dslots = dbt[:, (L - 1) // bs].long() * bs + (L - 1) % bs
    n_parts = ops.decode_num_parts(B, nkv, L)
    ws = ops.decode_workspace(B, nq, D, n_parts, dev)
    dmeta = AttnMeta(False, dpos, dslots, dbt, dctx, n_parts=n_parts, workspace=ws)
    # prefill rows: P prompts of C new tokens (no cached prefix)
    pbt = (1 + B * nb_d + torch.arange(P * nb_p, device=dev, dtype=torch.int32)).view(P, nb_p)
    ppos = torch.arange(C, device=dev, dtype=torch.int64).repeat(P)
    pslots = torch.cat([pbt[i].long()[torch.arange(C, device=dev) // bs] * bs + torch.arange(C, device=dev) % bs
                        for i in range(P)])
    cu = torch.arange(0, P * C + 1, C, device=dev, dtype=torch.int32)
    pctx = torch.full((P,), C, device=dev, dtype=torch.int32)
    work = torch.tensor(ops.prefill_work_list([C] * P, [C] * P, nq, nkv), dtype=torch.int32, device=dev)
    plog = cu[1:].long() - 1
    pmeta = AttnMeta(True, ppos, pslots, pbt, pctx, logits_idx=plog, cu_seqlens_q=cu, work=work)
    # the fused mixed step of today's engine
    fmeta = AttnMeta(True, torch.cat([ppos, dpos]), torch.cat([pslots, dslots]), pbt, pctx,
                     logits_idx=torch.cat([plog, torch.arange(P * C, P * C + B, device=dev)]), cu_seqlens_q=cu,
                     work=work, num_prefill_tokens=P * C, decode=dmeta)
    pids = torch.randint(0, cfg.vocab_size, (P * C,), device=dev)
    dids = torch.randint(0, cfg.vocab_size, (B,), device=dev)
    fids = torch.cat([pids, dids])

    # decode step as a hipGraph (the engine replays one per batch bucket)
    side = torch.cuda.Stream(dev)
    m.forward(dids, dmeta, caches)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        m.forward(dids, dmeta, caches)
    torch.cuda.synchronize()

    def fused():
        m.forward(fids, fmeta, caches)

    def prefill():
        m.forward(pids, pmeta, caches)

    def decode():
        g.replay()

    def serial():
        m.forward(pids, pmeta, caches)
        g.replay()

    main_s = torch.cuda.current_stream(dev)

    def split():
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            g.replay()
        m.forward(pids, pmeta, caches)
        main_s.wait_stream(side)

    res = {"shape": {"prompts": P, "chunk": C, "decode": B, "ctx": L}}
    for _ in range(2):  # interleaved rounds
        for name, fn in (("fused", fused), ("prefill", prefill), ("decode", decode), ("serial", serial),
                         ("split", split)):
            res.setdefault(name, []).append(timed(fn))
        print(json.dumps(res), flush=True)
    best = {k: min(v) for k, v in res.items() if k != "shape"}
    best["split_vs_fused"] = round(best["split"] / best["fused"], 3)
    best["decode_hidden_frac"] = round((best["serial"] - best["split"]) / best["decode"], 3)
    print(json.dumps(best), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"runs": res, "best_ms": best}, f, indent=1)


if __name__ == "__main__":
    main()
