"""Per-token cost of a prefill forward vs its token count (Llama-3-8B, random
weights, one MI355X): are small mixed steps (the ~1000-token remainder of a
prompt split by the step budget) and steps of awkward size (5-7k tokens,
partly filled GEMM tile rounds) much dearer per token than full 8192-token
steps?  T tokens as T / 512 prompts of 512 new tokens (no cached context) so
attention stays a small, linear share; the warm-up GEMM tuners run first,
as in the engine.

  python -m tools.forward_size_probe [--out profiles/...]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from dynamo_exp_amd import ops  # noqa: E402
from dynamo_exp_amd.models.config import get_config  # noqa: E402
from dynamo_exp_amd.models.llama import AttnMeta, LlamaForCausalLM  # noqa: E402


@torch.inference_mode()
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--sizes", default="1024,1536,2048,3072,4096,5120,5632,6144,7168,8192")
    ap.add_argument("--seg", type=int, default=512)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = get_config("llama3-8b")
    m = LlamaForCausalLM(cfg, device=dev).random_init(1)
    sizes = [int(s) for s in a.sizes.split(",")]
    m.enable_fused_mlp()
    m.tune_prefill_gemms(max(sizes) + 128)  # as the engine: buckets from 2048 tokens
    bs, S = 64, a.seg
    nkv, D = m.n_kv, m.head_dim
    nb = -(-S // bs)
    P_max = max(sizes) // S
    kv = torch.zeros(cfg.num_hidden_layers, 2, P_max * nb + 1, nkv, bs, D, device=dev, dtype=torch.bfloat16)
    caches = [(kv[i, 0], kv[i, 1]) for i in range(cfg.num_hidden_layers)]
    rows = []
    for T in sizes:
        P = T // S
        bt = (1 + torch.arange(P * nb, device=dev, dtype=torch.int32)).view(P, nb)
        pos = torch.arange(S, device=dev, dtype=torch.int64).repeat(P)
        slots = (bt.long()[:, torch.arange(S, device=dev) // bs] * bs + torch.arange(S, device=dev) % bs).reshape(-1)
        cu = torch.arange(0, P * S + 1, S, device=dev, dtype=torch.int32)
        ctx = torch.full((P,), S, device=dev, dtype=torch.int32)
        work = torch.tensor(ops.prefill_work_list([S] * P, [S] * P, m.n_q, nkv), dtype=torch.int32, device=dev)
        meta = AttnMeta(True, pos, slots, bt, ctx, logits_idx=cu[1:].long() - 1, cu_seqlens_q=cu, work=work)
        ids = torch.randint(0, cfg.vocab_size, (P * S,), device=dev)
        for _ in range(2):
            m.forward(ids, meta, caches)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(3):
            e0.record()
            for _ in range(3):
                m.forward(ids, meta, caches)
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) / 3)
        r = {"tokens": P * S, "ms": round(best, 3), "us_per_token": round(best * 1e3 / (P * S), 3)}
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.out:
        with open(a.out, "w") as f:
            f.write("# tools/forward_size_probe.py: Llama-3-8B prefill forward (prompts of 512 new tokens) vs token count\n")
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
