"""Greedy tokens of an fp8-KV engine vs a bf16-KV engine on the same weights
(tests/test_kv_fp8.py::test_engine_fp8_kv_gpu) under both prefill-attention
variants (ops.PREFILL_WAVES 91 / 92): is a first-token difference the
e4m3 cache or the attention loop?"""
import sys

import torch

sys.path.insert(0, ".")
from dynamo_exp_amd import ops  # noqa: E402
from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine  # noqa: E402
from dynamo_exp_amd.engine.request import SamplingParams  # noqa: E402


def gen(eng, prompts, n):
    out = {}
    for i, p in enumerate(prompts):
        eng.add_request(f"q{i}", p, SamplingParams(max_tokens=n, ignore_eos=True),
                        on_output=lambda r, t, lp, fin: out.setdefault(r.request_id, []).extend(t))
    while eng.has_unfinished():
        eng.step()
    return [out[f"q{i}"] for i in range(len(prompts))]


prompts = [list(range(10 + i, 300 + 41 * i)) for i in range(6)]
kw = dict(model="small", device="cuda:0", block_size=64, max_model_len=2048, num_gpu_blocks=256, max_num_seqs=8,
          graph_sizes=(1, 2, 4, 8), max_num_batched_tokens=512)
res = {}
for v in (92, 91):
    ops.PREFILL_WAVES = v
    e8 = LLMEngine(EngineConfig(kv_cache_dtype="fp8", **kw))
    e8.warmup()
    eb = LLMEngine(EngineConfig(**kw), model=e8.model)
    eb.warmup()
    a, b = gen(e8, prompts, 12), gen(eb, prompts, 12)
    res[v] = {"first_same": sum(x[0] == y[0] for x, y in zip(a, b)),
              "same": sum(p == q for x, y in zip(a, b) for p, q in zip(x, y)), "bf16": b}
    del e8, eb
    torch.cuda.empty_cache()
print({v: (r["first_same"], r["same"]) for v, r in res.items()})
print("bf16 tokens identical across variants:", res[91]["bf16"] == res[92]["bf16"])
