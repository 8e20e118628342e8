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

  split_cu -- split, with the two streams on disjoint CU sets (hipExtStreamCreateWithCUMask:
             --side-cus CUs for the decode graph, the rest for the prefill forward; run with
             DX_GEMM256_CUS = the prefill stream's CU count so the persistent GEMM grid fits it)
  gemm_cu  -- one prefill-size GEMM on the masked prefill stream vs the full chip (power-capped
             GEMMs may lose little with fewer CUs)

  python -m tools.mixed_split_probe [--out profiles/...] [--side-cus 32]
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
    ap.add_argument("--side-cus", type=int, default=0)
    ap.add_argument("--mask", default="xcd", help="tail | stride | xcd | mod8:<r>,<r>.. (side = CUs i with i % 8 in r)")
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

    variants = [("fused", fused), ("prefill", prefill), ("decode", decode), ("serial", serial), ("split", split)]
    if a.side_cus:
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
        per = n_cu // 8  # CUs per XCD (mask bit i = CU i; XCD = i // per, measured: a contiguous
        # 32-CU tail costs the prefill GEMMs a whole XCD)
        if a.mask == "tail":
            side_set = set(range(n_cu - a.side_cus, n_cu))
        elif a.mask == "stride":
            side_set = set(range(7, n_cu, max(1, n_cu // a.side_cus)))
        elif a.mask.startswith("mod8:"):
            rs = {int(r) for r in a.mask[5:].split(",")}
            side_set = {c for c in range(n_cu) if c % 8 in rs}
        else:  # the top side_cus / 8 CUs of every XCD
            k = a.side_cus // 8
            side_set = {x * per + per - 1 - j for x in range(8) for j in range(k)}

        def masked(cus):
            words = [0] * ((n_cu + 31) // 32)
            for c in cus:
                words[c // 32] |= 1 << (c % 32)
            arr = (ctypes.c_uint32 * len(words))(*words)
            h = ctypes.c_void_p()
            rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), arr)
            assert rc == 0, rc
            return torch.cuda.ExternalStream(h.value, device=dev)

        s_main, s_side = masked(sorted(set(range(n_cu)) - side_set)), masked(sorted(side_set))
        gs = torch.cuda.CUDAGraph()  # the decode step captured on the side stream
        with torch.cuda.graph(gs, stream=s_side):
            m.forward(dids, dmeta, caches)
        torch.cuda.synchronize()

        def split_cu():
            cur = torch.cuda.current_stream(dev)
            s_main.wait_stream(cur)
            s_side.wait_stream(cur)
            with torch.cuda.stream(s_side):
                gs.replay()
            with torch.cuda.stream(s_main):
                m.forward(pids, pmeta, caches)
            cur.wait_stream(s_main)
            cur.wait_stream(s_side)

        wx = torch.randn(P * C, 14336, device=dev, dtype=torch.bfloat16)
        ww = [torch.randn(4096, 14336, device=dev, dtype=torch.bfloat16) for _ in range(4)]

        def gemm_full():
            for w in ww:
                torch.matmul(wx, w.t())

        def gemm_cu():
            cur = torch.cuda.current_stream(dev)
            s_main.wait_stream(cur)
            with torch.cuda.stream(s_main):
                for w in ww:
                    torch.matmul(wx, w.t())
            cur.wait_stream(s_main)

        variants += [("split_cu", split_cu), ("gemm_full", gemm_full), ("gemm_cu", gemm_cu)]
    res = {"shape": {"prompts": P, "chunk": C, "decode": B, "ctx": L, "side_cus": a.side_cus, "mask": a.mask}}
    for _ in range(2):  # interleaved rounds
        for name, fn in variants:
            res.setdefault(name, []).append(timed(fn))
        print(json.dumps(res), flush=True)
    best = {k: min(v) for k, v in res.items() if k != "shape"}
    best["split_vs_fused"] = round(best["split"] / best["fused"], 3)
    if a.side_cus:
        best["split_cu_vs_fused"] = round(best["split_cu"] / best["fused"], 3)
        best["gemm_cu_vs_full"] = round(best["gemm_cu"] / best["gemm_full"], 3)
    best["decode_hidden_frac"] = round((best["serial"] - best["split"]) / best["decode"], 3)
    print(json.dumps(best), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"runs": res, "best_ms": best}, f, indent=1)


if __name__ == "__main__":
    main()
