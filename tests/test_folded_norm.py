"""Folded RMSNorm (models/llama.py fold_norms / _forward_folded): the norm
weights folded into the qkv / gate_up weight columns, the residual adds run
as the o / down GEMMs' accumulation, and the 1 / rms row scale applied by the
consumers (rope_cache, the fused SwiGLU GEMM's epilogue).

* kernels vs plain fp32 PyTorch references (GPU): row_rrms, rope_cache with a
  row scale (Q in the row, K / V in the cache), gemm256's SwiGLU epilogue
  with a row scale;
* the model: an engine on the folded forward decodes the tokens of an
  engine on the unfused forward of the same weights, with non-trivial norm
  weights (CPU: exact tiny model; GPU: Llama-3-8B@4 layers, near-ties allowed).
"""
import copy
import os

import pytest
import torch

from dynamo_exp_amd import ops
from dynamo_exp_amd.ops import reference as ref


def _rel(got, want):
    return ((got.float() - want.float()).abs().max() / want.float().abs().max()).item()


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 300, 8192])
def test_row_rrms_gpu(cuda, M):
    torch.manual_seed(M)
    x = (torch.randn(M, 4096, device=cuda) * 3).bfloat16()
    got = ops.row_rrms(x, 1e-5)
    want = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)
    assert got.dtype == torch.float32 and got.shape == (M,)
    assert _rel(got, want) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("M", [128, 3000])
def test_gemm256_silu_row_scale_gpu(cuda, M):
    torch.manual_seed(7 + M)
    K, F = 4096, 1024
    x = (torch.rand(M, K, device=cuda) * 2 - 1).bfloat16()
    w = (torch.randn(2 * F, K, device=cuda) / 64).bfloat16()
    rs = torch.rand(M, device=cuda) * 2 + 0.1
    wi = ref.interleave_gate_up(w, ops.GEMM256_BLK).contiguous()
    got = ops.gemm256(x, wi, ops.GEMM256_EPI_SILU, row_scale=rs)
    gu = (x.float() @ w.float().t()) * rs[:, None]
    want = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    assert _rel(got, want) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("rotate_q", [True, False])
def test_rope_cache_row_scale_gpu(cuda, rotate_q):
    torch.manual_seed(3)
    Hq, Hkv, D, bs, T = 8, 2, 128, 16, 45
    qkv = (torch.randn(T, (Hq + 2 * Hkv) * D, device=cuda)).bfloat16()
    rs = torch.rand(T, device=cuda) + 0.5
    pos = torch.arange(7, 7 + T, device=cuda)
    cos_sin = ref.rope_cos_sin(D, 4096, 500000.0).to(cuda)
    slots = torch.arange(T, device=cuda, dtype=torch.int64) + 3
    caches = [(torch.zeros(8, Hkv, bs, D, device=cuda).bfloat16(), torch.zeros(8, Hkv, bs, D, device=cuda).bfloat16())
              for _ in range(2)]
    want_row = (qkv.float() * rs[:, None]).bfloat16()
    ops.rope_cache(want_row, pos, cos_sin, slots, caches[0][0], caches[0][1], Hq, Hkv, D, bs, rotate_q=rotate_q)
    got_row = qkv.clone()
    ops.rope_cache(got_row, pos, cos_sin, slots, caches[1][0], caches[1][1], Hq, Hkv, D, bs, rotate_q=rotate_q,
                   row_scale=rs)
    torch.cuda.synchronize()
    # Q (what attention reads) and the cache, scaled then rotated
    assert _rel(got_row[:, :Hq * D], want_row[:, :Hq * D]) < 1e-2
    for a, b in zip(caches[1], caches[0]):
        assert _rel(a, b) < 1e-2


def _engines(device, model_name, max_len, blocks, seed=3):
    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
    from dynamo_exp_amd.models.config import get_config
    from dynamo_exp_amd.models.llama import LlamaForCausalLM

    dev = torch.device(device)
    base = LlamaForCausalLM(get_config(model_name), device=dev).random_init(seed)
    g = torch.Generator().manual_seed(11)
    for L in base.layers:  # non-trivial norm weights: the fold must carry them
        for n in ("ln1", "ln2"):
            L[n] = (1.0 + 0.2 * torch.randn(L[n].shape, generator=g)).to(L[n].dtype).to(dev)
    other = copy.deepcopy(base)
    kw = dict(model=model_name, device=device, block_size=16 if device == "cpu" else 64, max_model_len=max_len,
              num_gpu_blocks=blocks, max_num_seqs=8, seed=seed, use_cuda_graph=False, chunked_prefill=False,
              max_num_batched_tokens=4096)
    old = os.environ.get("DX_FOLD_NORM")
    os.environ["DX_FOLD_NORM"] = "0"
    try:
        plain = LLMEngine(EngineConfig(**kw), model=base)
    finally:
        if old is None:
            del os.environ["DX_FOLD_NORM"]
        else:
            os.environ["DX_FOLD_NORM"] = old
    folded = LLMEngine(EngineConfig(**kw), model=other)
    assert folded.model.norm_folded and not plain.model.norm_folded
    return plain, folded


def _run(eng, prompts, n):
    from dynamo_exp_amd.engine.request import SamplingParams

    out = {}
    for rid, p in prompts.items():
        eng.add_request(rid, p, SamplingParams(max_tokens=n, ignore_eos=True),
                        on_output=lambda r, t, lp, fin: out.setdefault(r.request_id, []).extend(zip(t, lp)))
    while eng.has_unfinished():
        eng.step()
    return out


def test_folded_forward_matches_unfused_cpu():
    plain, folded = _engines("cpu", "tiny", 512, 200)
    folded.model.fold_min_m = 1  # every forward on the folded path (prefill and decode)
    prompts = {f"r{i}": [(5 * i + 3 * j) % 500 + 1 for j in range(60 + 13 * i)] for i in range(3)}
    want = _run(plain, prompts, 6)
    got = _run(folded, prompts, 6)
    for rid in prompts:
        assert [t for t, _ in got[rid]] == [t for t, _ in want[rid]], rid
        for (_, a), (_, b) in zip(got[rid], want[rid]):
            assert abs(a - b) < 2e-2, (rid, a, b)


@pytest.mark.gpu
def test_folded_forward_matches_unfused_gpu(cuda):
    """Prompts of 1000-1300 tokens (the folded path at M >= 512, the unfused
    path below) on Llama-3-8B@4 layers; greedy tokens equal or near-tie
    swaps (different rounding points on random weights)."""
    plain, folded = _engines(str(cuda), "llama3-8b@4", 2048, 256)
    assert folded.model.gu_blk  # the fused SwiGLU epilogue with the row scale runs
    g = torch.Generator().manual_seed(5)
    prompts = {f"r{i}": torch.randint(1, 120000, (1000 + 97 * i,), generator=g).tolist() for i in range(4)}
    want = _run(plain, prompts, 8)
    got = _run(folded, prompts, 8)
    same = 0
    for rid, w in want.items():
        gt = got[rid]
        if [t for t, _ in gt] == [t for t, _ in w]:
            same += 1
            continue
        j = next(k for k, (a, b) in enumerate(zip(gt, w)) if a[0] != b[0])
        assert abs(gt[j][1] - w[j][1]) < 0.1, (rid, j, gt[j], w[j])
    assert same >= len(prompts) // 2, same
    # the first token's logprob (the prefill forward) agrees closely
    for rid in prompts:
        assert abs(got[rid][0][1] - want[rid][0][1]) < 0.05, rid
