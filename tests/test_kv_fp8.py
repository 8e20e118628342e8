"""FP8 (OCP e4m3fn) KV cache, kv_cache_dtype="fp8": the cache write (rope +
quantize in csrc/kernels/rope_cache.hip), decode attention dequantizing on
load, prefill attention through the bf16 dequant scratch, and the engine end
to end -- each against a PyTorch reference of the same op (fp32 math over the
identical e4m3 values), plus the CPU reference path."""
import math

import pytest
import torch

from dynamo_exp_amd import ops
from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
from dynamo_exp_amd.engine.request import SamplingParams
from dynamo_exp_amd.ops import reference as ref

FP8 = torch.float8_e4m3fn


def _gen(eng, prompts, n):
    out = {}
    for i, p in enumerate(prompts):
        eng.add_request(f"q{i}", p, SamplingParams(max_tokens=n, ignore_eos=True),
                        on_output=lambda r, t, lp, fin: out.setdefault(r.request_id, []).extend(t))
    while eng.has_unfinished():
        eng.step()
    return [out[f"q{i}"] for i in range(len(prompts))]


def test_to_cache_clamps_and_scales_cpu():
    x = torch.tensor([1000.0, -3.0, 0.3])
    q = ref.to_cache(x, FP8, 2.0)
    assert q.dtype == FP8 and not torch.isnan(q.float()).any()
    torch.testing.assert_close(q.float(), torch.tensor([448.0, -1.5, 0.15625]))


def test_engine_fp8_kv_cpu():
    """The CPU reference path runs the fp8 cache end to end (KV bytes halved)
    and its greedy tokens mostly agree with the bf16 cache on random weights."""
    prompts = [list(range(5 + i, 60 + 9 * i)) for i in range(3)]
    kw = dict(model="tiny", device="cpu", block_size=16, max_model_len=256, num_gpu_blocks=64, max_num_seqs=4,
              use_cuda_graph=False)
    e8 = LLMEngine(EngineConfig(kv_cache_dtype="fp8", **kw))
    eb = LLMEngine(EngineConfig(**kw), model=e8.model)
    assert e8.runner.kv_cache.dtype == FP8 and e8.runner.kv_bytes * 2 == eb.runner.kv_bytes
    a, b = _gen(e8, prompts, 6), _gen(eb, prompts, 6)
    assert all(len(x) == 6 for x in a)
    same = sum(x == y for ra, rb in zip(a, b) for x, y in zip(ra, rb))
    assert same >= 12, (a, b)  # e4m3 K/V move logits by a few %: allow near-tie flips
    with pytest.raises(ValueError):
        LLMEngine(EngineConfig(kv_cache_dtype="int4", **kw))


def _paged_fp8(cuda, seq_lens, hkv, bs, scales, seed=0, hd=128):
    torch.manual_seed(seed)
    nb = sum((s + bs - 1) // bs for s in seq_lens) + 3
    kb = torch.randn(nb, hkv, bs, hd) * 3
    vb = torch.randn(nb, hkv, bs, hd) * 3
    kc, vc = ref.to_cache(kb, FP8, scales[0]), ref.to_cache(vb, FP8, scales[1])
    perm = torch.randperm(nb).tolist()
    bt = torch.zeros(len(seq_lens), max((s + bs - 1) // bs for s in seq_lens) + 1, dtype=torch.int32)
    i = 0
    for b, s in enumerate(seq_lens):
        for j in range((s + bs - 1) // bs):
            bt[b, j] = perm[i]
            i += 1
    return kc.to(cuda), vc.to(cuda), bt.to(cuda)


@pytest.mark.gpu
def test_rope_cache_fp8_gpu(cuda):
    hq, hkv, hd, bs, T = 32, 8, 128, 16, 50
    torch.manual_seed(3)
    qkv = (torch.randn(T, (hq + 2 * hkv) * hd) * 4).to(torch.bfloat16).to(cuda)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int64).to(cuda)
    cos_sin = ref.rope_cos_sin(hd, 8192, 500000.0).to(cuda)
    slots = torch.randperm(8 * bs)[:T].to(cuda)
    scales = (0.5, 2.0)
    kc = torch.zeros(8, hkv, bs, hd, dtype=FP8, device=cuda)
    vc = torch.zeros_like(kc)
    q1 = qkv.clone()
    ops.rope_cache(q1, pos, cos_sin, slots, kc, vc, hq, hkv, hd, bs, kv_scales=scales)
    kr, vr = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q2 = qkv.cpu().clone()
    ref.rope_cache(q2, pos.cpu(), cos_sin.cpu(), slots.cpu(), kr, vr, hq, hkv, hd, bs, kv_scales=scales)
    torch.testing.assert_close(q1.cpu().float(), q2.float(), atol=2e-2, rtol=2e-2)
    # same e4m3 codes up to one ulp where the bf16 rope rounding differs
    for got, want, s in ((kc, kr, scales[0]), (vc, vr, scales[1])):
        g, w = got.cpu().float(), want.float()
        assert (g - w).abs().max().item() <= 0.13 * w.abs().max().item()
        assert (g == w).float().mean().item() > 0.97


@pytest.mark.gpu
@pytest.mark.parametrize("hq,hkv", [(32, 8), (16, 2), (8, 8)])
def test_decode_attention_fp8_gpu(cuda, hq, hkv, monkeypatch):
    seq_lens = [1, 17, 64, 333, 1500, 4100]
    bs, scales = 64, (0.5, 2.0)
    kc, vc, bt = _paged_fp8(cuda, seq_lens, hkv, bs, scales)
    B = len(seq_lens)
    q = torch.randn(B, hq, 128, device=cuda, dtype=torch.bfloat16)
    ctx = torch.tensor(seq_lens, dtype=torch.int32, device=cuda)
    sc = 1 / math.sqrt(128)
    want = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), torch.arange(B + 1, dtype=torch.int32),
                               ctx.cpu(), sc, bs, scales)
    # 4 / 8 query heads per KV head take the MFMA kernel by default: both kernels checked
    for mfma in ("1", "0"):
        monkeypatch.setenv("DX_DECODE_MFMA", mfma)
        for n_parts in (1, 3, 7):
            out = torch.empty_like(q)
            ops.decode_attention(q, kc, vc, bt, ctx, sc, out, n_parts, kv_scales=scales)
            err = (out.float().cpu() - want.float()).abs().max().item()
            assert err < 0.03 * want.abs().max().item() + 0.02, (mfma, n_parts, err)


@pytest.mark.gpu
def test_prefill_attention_fp8_gpu(cuda):
    hq, hkv, bs, scales = 32, 8, 64, (0.5, 2.0)
    cases = [(37, 37), (100, 164), (1, 1), (300, 300), (64, 640), (130, 3131)]
    ctx_list = [c for _, c in cases]
    kc, vc, bt = _paged_fp8(cuda, ctx_list, hkv, bs, scales, seed=1)
    qlens = [q for q, _ in cases]
    T = sum(qlens)
    cu = torch.tensor([0] + torch.tensor(qlens).cumsum(0).tolist(), dtype=torch.int32)
    q = torch.randn(T, hq, 128, device=cuda, dtype=torch.bfloat16)
    ctx = torch.tensor(ctx_list, dtype=torch.int32)
    sc = 1 / math.sqrt(128)
    out = torch.empty_like(q)
    ops.prefill_attention(q, kc, vc, bt, cu.to(cuda), ctx.to(cuda), sc, out, kv_scales=scales)
    want = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), cu, ctx, sc, bs, scales)
    err = (out.float().cpu() - want.float()).abs().max().item()
    assert err < 0.03 * want.abs().max().item() + 0.02, err


@pytest.mark.gpu
def test_engine_fp8_kv_gpu(cuda):
    """Graph decode + chunked prefill with the fp8 cache: tokens close to the
    bf16-cache engine on the same weights (e4m3 K/V: near-tie flips allowed),
    and the CPU fp8 reference decides the first token identically."""
    prompts = [list(range(10 + i, 300 + 41 * i)) for i in range(6)]
    kw = dict(model="small", device="cuda:0", block_size=64, max_model_len=2048, num_gpu_blocks=256, max_num_seqs=8,
              graph_sizes=(1, 2, 4, 8), max_num_batched_tokens=512)
    e8 = LLMEngine(EngineConfig(kv_cache_dtype="fp8", **kw))
    e8.warmup()
    eb = LLMEngine(EngineConfig(**kw), model=e8.model)
    eb.warmup()
    a, b = _gen(e8, prompts, 12), _gen(eb, prompts, 12)
    first_same = sum(ra[0] == rb[0] for ra, rb in zip(a, b))
    same = sum(x == y for ra, rb in zip(a, b) for x, y in zip(ra, rb))
    assert first_same >= 5 and same >= 0.6 * 72, (a, b)


def test_calibrate_kv_scales_cpu():
    """Calibrated scales map the observed |K| / |V| maxima onto e4m3's range,
    and the engine keeps generating with them."""
    kw = dict(model="tiny", device="cpu", block_size=16, max_model_len=256, num_gpu_blocks=64, max_num_seqs=4,
              use_cuda_graph=False)
    e8 = LLMEngine(EngineConfig(kv_cache_dtype="fp8", **kw))
    prompts = [list(range(3 + i, 40 + 7 * i)) for i in range(3)]
    ks, vs = e8.calibrate_kv_scales(prompts)
    assert 0 < ks and 0 < vs and e8.model.kv_scales == (ks, vs) and e8.model.kv_amax is None
    assert not e8.has_unfinished() and e8.kv.num_free() > 0
    out = _gen(e8, prompts[:2], 4)
    assert all(len(o) == 4 for o in out)
    with pytest.raises(ValueError):
        LLMEngine(EngineConfig(**kw)).calibrate_kv_scales(prompts)



def test_calibrate_refused_once_a_transfer_agent_is_attached_cpu():
    """peers cache an engine's published kv_scales, so new scales
    after a KVTransferAgent attached would decode its bytes wrongly."""
    from dynamo_exp_amd.disagg.agent import KVTransferAgent
    from dynamo_exp_amd.disagg.transfer import LoopbackHub, LoopbackLinks

    kw = dict(model="tiny", device="cpu", block_size=16, max_model_len=256, num_gpu_blocks=32, max_num_seqs=2,
              use_cuda_graph=False, kv_cache_dtype="fp8")
    e = LLMEngine(EngineConfig(**kw))
    KVTransferAgent(e, None, "p", "t", links=LoopbackLinks(LoopbackHub("cpu"), "p"))
    with pytest.raises(RuntimeError, match="before attaching"):
        e.calibrate_kv_scales([list(range(3, 40))])


def test_calibrated_engine_matches_fresh_engine_with_those_scales_cpu():
    """blocks written during (or before) calibration hold
    bytes quantised with the old scales; after calibrating, the same prompts
    with prefix caching on must decode exactly what a fresh engine built with
    the calibrated scales decodes (no stale-scale prefix hits), and the router
    saw the stale blocks Removed."""
    kw = dict(model="tiny", device="cpu", block_size=16, max_model_len=256, num_gpu_blocks=64, max_num_seqs=4,
              use_cuda_graph=False, kv_cache_dtype="fp8")
    e8 = LLMEngine(EngineConfig(**kw))
    events = []
    e8.add_kv_event_listener(lambda evs: events.extend(evs))
    prompts = [list(range(3 + i, 70 + 7 * i)) for i in range(3)]
    _gen(e8, prompts[:1], 2)  # served before calibration: cached at scale 1.0
    scales = e8.calibrate_kv_scales(prompts)
    assert scales != (1.0, 1.0)
    stored = {e.seq_hash for e in events if e.kind == "stored"}
    removed = {e.seq_hash for e in events if e.kind == "removed"}
    assert stored and stored <= removed  # every old-scale block was withdrawn from the router
    assert e8.kv.prefix_hit_tokens_for(prompts[0]) == 0
    fresh = LLMEngine(EngineConfig(kv_scales=scales, **kw), model=e8.model)
    assert _gen(e8, prompts, 6) == _gen(fresh, prompts, 6)


def test_kv_scale_mismatch_refused_by_transfer_metadata_cpu():
    """two fp8 workers whose kv_scales differ must not
    exchange raw e4m3 bytes."""
    import json

    from dynamo_exp_amd.disagg.agent import KVTransferAgent
    from dynamo_exp_amd.disagg.transfer import LoopbackHub, LoopbackLinks

    kw = dict(model="tiny", device="cpu", block_size=16, max_model_len=256, num_gpu_blocks=32, max_num_seqs=2,
              use_cuda_graph=False, kv_cache_dtype="fp8")
    a = LLMEngine(EngineConfig(kv_scales=(0.5, 0.25), **kw))
    b = LLMEngine(EngineConfig(**kw))  # uncalibrated: scales (1, 1)

    class CP:
        kv = {}

        def call(self, name, *args, **kw):
            if name == "put":
                self.kv[args[0]] = args[1]
            return self.kv.get(args[0])

    hub = LoopbackHub("cpu")
    cp = CP()
    pa = KVTransferAgent(a, cp, "p", "t", links=LoopbackLinks(hub, "p")).start_sync()
    da = KVTransferAgent(b, cp, "d", "t", links=LoopbackLinks(hub, "d")).start_sync()
    assert json.loads(cp.kv["t/kv_transfer/p/0"])["kv_scales"] == [0.5, 0.25]
    with pytest.raises(RuntimeError, match="kv_scales"):
        pa.meta_of("d")
    with pytest.raises(RuntimeError, match="kv_scales"):
        da.meta_of("p")


def test_fp8_scratch_plan_packs_and_caps_cpu():
    """the fp8 prefill dequant scratch holds only live
    context blocks (sum of ceil(ctx / bs)), in groups under the cap."""
    groups = ops.fp8_scratch_plan([100, 64, 3000, 5], 64, 60, 50)
    assert [(g[0], g[1], g[2]) for g in groups] == [(0, 3, 50), (3, 4, 1)]
    s0, s1, n, tab = groups[0]
    assert tab[0, :2].tolist() == [0, 1] and tab[1, 0] == 2 and tab[2, :47].tolist() == list(range(3, 50))
    assert all(g[2] <= 50 for g in groups)


@pytest.mark.gpu
def test_fp8_prefill_scratch_groups_match_single_pass_gpu(cuda):
    """A prefill batch whose fp8 context exceeds the scratch cap runs its
    attention in sequence groups: same tokens as one pass under a large cap,
    and the scratch never exceeds the cap."""
    prompts = [list(range(10 + i, 700 + 37 * i)) for i in range(5)]
    kw = dict(model="small", device="cuda:0", block_size=64, max_model_len=2048, num_gpu_blocks=256, max_num_seqs=8,
              use_cuda_graph=False, max_num_batched_tokens=8192, chunked_prefill=False, kv_cache_dtype="fp8")
    a = LLMEngine(EngineConfig(**kw))
    b = LLMEngine(EngineConfig(**kw), model=a.model)
    b.runner.fp8_scratch_cap = 16  # ~1-2 prompts per group
    want, got = _gen(a, prompts, 6), _gen(b, prompts, 6)
    assert got == want
    ws = [v for k, v in ops._KV_SCRATCH.items()]
    assert ws and min(w[0].shape[0] for w in ws) >= 16
