"""Numerics of the gfx950 HIP kernels vs plain-PyTorch fp32 references.

Every test runs the HIP kernel (``dynamo_exp_amd._C_kernels``; the ops raise
if it is missing on a GPU box) and compares with :mod:`dynamo_exp_amd.ops.reference`.
"""
import math

import os

import pytest
import torch

from dynamo_exp_amd import ops
from dynamo_exp_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    lim = atol + rtol * b.abs().max().item()
    assert err <= lim, f"{msg} max abs err {err} > {lim}"


def test_native_loaded(cuda):
    from dynamo_exp_amd import _native

    m = _native.kernels()
    assert m.arch == "gfx950"


@pytest.mark.parametrize("hidden", [4096, 8192, 1000 * 8])
@pytest.mark.parametrize("rows", [1, 7, 64])
def test_rmsnorm(cuda, rows, hidden):
    torch.manual_seed(0)
    x = torch.randn(rows, hidden, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(hidden, device=cuda, dtype=torch.bfloat16)
    out = ops.rmsnorm(x, w, 1e-5)
    _close(out, ref.rmsnorm(x.cpu(), w.cpu(), 1e-5), 0.05, 0.01, "rmsnorm")
    r = torch.randn_like(x)
    r_ref = r.clone().cpu()
    y = ops.add_rmsnorm(x, r, w, 1e-5)
    y_ref = ref.add_rmsnorm(x.cpu(), r_ref, w.cpu(), 1e-5)
    _close(r, r_ref, 0.02, 0.01, "residual")
    _close(y, y_ref, 0.05, 0.01, "add_rmsnorm")


def _paged_setup(cuda, seq_lens, hkv, hd=128, bs=16, nb_extra=3, seed=0):
    torch.manual_seed(seed)
    nb_needed = sum((s + bs - 1) // bs for s in seq_lens)
    nb = nb_needed + nb_extra
    kc = torch.randn(nb, hkv, bs, hd, device=cuda, dtype=torch.bfloat16)
    vc = torch.randn(nb, hkv, bs, hd, device=cuda, dtype=torch.bfloat16)
    perm = torch.randperm(nb).tolist()
    maxb = max((s + bs - 1) // bs for s in seq_lens)
    bt = torch.zeros(len(seq_lens), maxb + 1, dtype=torch.int32)
    i = 0
    for b, s in enumerate(seq_lens):
        for j in range((s + bs - 1) // bs):
            bt[b, j] = perm[i]
            i += 1
    return kc, vc, bt.to(cuda)


@pytest.mark.parametrize("hq,hkv", [(32, 8), (16, 2), (8, 8), (8, 4), (64, 8), (32, 2)])
@pytest.mark.parametrize("bs", [16, 32, 64])
def test_decode_attention(cuda, hq, hkv, bs, monkeypatch):
    seq_lens = [1, 17, 64, 333, 1500, 4100]
    kc, vc, bt = _paged_setup(cuda, seq_lens, hkv, bs=bs)
    # stale cache bytes past each context in its last block are NaN: masked
    # rows must not reach the output (P = 0 times NaN)
    for b, s in enumerate(seq_lens):
        if s % bs:
            blk = int(bt[b, s // bs])
            kc[blk, :, s % bs:] = float("nan")
            vc[blk, :, s % bs:] = float("nan")
    B = len(seq_lens)
    q = torch.randn(B, hq, 128, device=cuda, dtype=torch.bfloat16)
    ctx = torch.tensor(seq_lens, dtype=torch.int32, device=cuda)
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), torch.arange(B + 1, dtype=torch.int32),
                              ctx.cpu(), scale, bs)
    # the MFMA kernel runs by default (block size 16 too: two blocks per
    # 32-token chunk); both kernels are checked (the VALU kernel has no G = 16).  Balanced partitions: one part
    # per sequence (no reduce), a few, and more parts than some contexts have
    # chunks (empty trailing parts)
    for mfma in ("1", "0") if hq // hkv <= 8 else ("1",):
        monkeypatch.setenv("DX_DECODE_MFMA", mfma)
        for n_parts in (1, 3, 7, 40):
            out = torch.empty_like(q)
            ops.decode_attention(q, kc, vc, bt, ctx, scale, out, n_parts)
            _close(out, exp, 0.02, msg=f"decode mfma={mfma} n_parts={n_parts}")
    if ops.DECODE_TARGET_WGS == 512:
        assert ops.decode_num_parts(128, 8, 3214) == 1 and ops.decode_num_parts(32, 8, 3214) == 2
        assert ops.decode_num_parts(1, 8, 3214) == 13 and ops.decode_num_parts(8, 8, 16000) == 8


def test_decode_attention_padding_rows(cuda):
    """A captured decode graph's padding rows have context 0: with partitions (reduce kernel) and without, the
    real rows match the reference and the padding rows come out 0 (no division by a zero partition size)."""
    hq, hkv, bs = 32, 8, 64
    seq_lens = [700, 3100]
    kc, vc, bt = _paged_setup(cuda, seq_lens, hkv, bs=bs)
    bt = torch.cat([bt, torch.zeros(2, bt.shape[1], dtype=torch.int32, device=cuda)])
    q = torch.randn(4, hq, 128, device=cuda, dtype=torch.bfloat16)
    ctx = torch.tensor(seq_lens + [0, 0], dtype=torch.int32, device=cuda)
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q[:2].cpu(), kc.cpu(), vc.cpu(), bt[:2].cpu(), torch.arange(3, dtype=torch.int32),
                              ctx[:2].cpu(), scale, bs)
    for n_parts in (1, 4):
        out = torch.full_like(q, 7.0)
        ops.decode_attention(q, kc, vc, bt, ctx, scale, out, n_parts)
        _close(out[:2], exp, 0.02, msg=f"decode padding n_parts={n_parts}")
        if n_parts > 1:
            assert bool((out[2:] == 0).all()), "padding rows"


def test_decode_attention_strided_q(cuda):
    hq, hkv, hd, bs = 32, 8, 128, 16
    seq_lens = [5, 100, 700]
    kc, vc, bt = _paged_setup(cuda, seq_lens, hkv, bs=bs)
    B = len(seq_lens)
    qkv = torch.randn(B, (hq + 2 * hkv) * hd, device=cuda, dtype=torch.bfloat16)
    q = qkv[:, : hq * hd].view(B, hq, hd)
    ctx = torch.tensor(seq_lens, dtype=torch.int32, device=cuda)
    out = torch.empty(B, hq, hd, device=cuda, dtype=torch.bfloat16)
    ops.decode_attention(q, kc, vc, bt, ctx, 0.1, out, 2)
    exp = ref.paged_attention(q.cpu().contiguous(), kc.cpu(), vc.cpu(), bt.cpu(), torch.arange(B + 1, dtype=torch.int32),
                              ctx.cpu(), 0.1, bs)
    _close(out, exp, 0.02)


@pytest.fixture(params=[91, 92], ids=["v2", "v2-r3"])
def pa_variant(request):
    """Prefill-attention kernel variant (ops.PREFILL_WAVES): 91 = v2 (deferred
    rescale, static priority, widened epilogue), 92 = the round-3 loop kept
    for A/B (csrc/kernels/attn_prefill.hip)."""
    old = ops.PREFILL_WAVES
    ops.PREFILL_WAVES = request.param
    yield request.param
    ops.PREFILL_WAVES = old


@pytest.mark.parametrize("hq,hkv", [(32, 8), (16, 2), (8, 8), (8, 4)])
@pytest.mark.parametrize("bs", [16, 64])
def test_prefill_attention(cuda, hq, hkv, bs, pa_variant):
    # (q_len, ctx_len): pure prefill, prefix-cached, tiny, long
    cases = [(37, 37), (100, 164), (1, 1), (300, 300), (64, 640), (130, 131)]
    ctx_list = [c for _, c in cases]
    kc, vc, bt = _paged_setup(cuda, ctx_list, hkv, bs=bs, seed=1)
    qlens = [q for q, _ in cases]
    T = sum(qlens)
    cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0).tolist()), dtype=torch.int32)
    q = torch.randn(T, hq, 128, device=cuda, dtype=torch.bfloat16)
    ctx = torch.tensor(ctx_list, dtype=torch.int32)
    scale = 1 / math.sqrt(128)
    out = torch.empty_like(q)
    ops.prefill_attention(q, kc, vc, bt, cu.to(cuda), ctx.to(cuda), scale, out)
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), cu, ctx, scale, bs)
    _close(out, exp, 0.03, msg="prefill")


@pytest.mark.parametrize("cases", [[(3000, 3000)], [(1024, 3000), (2048, 2048)], [(512, 16384)],
                                   [(16384, 16384)]])
def test_prefill_attention_long(cuda, cases, pa_variant):
    """The headline shapes: ISL-3000 prompts (whole and as a chunk behind a
    cached prefix) and 16K contexts (a 512-token chunk at the end of 16K, and
    a whole 16K prompt), GQA 32/8, block 64 -- vs the fp32 reference on a
    subset of query rows (the full 16K^2 CPU reference is too slow)."""
    hq, hkv, bs = 32, 8, 64
    ctx_list = [c for _, c in cases]
    kc, vc, bt = _paged_setup(cuda, ctx_list, hkv, bs=bs, seed=4)
    qlens = [q for q, _ in cases]
    T = sum(qlens)
    cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0).tolist()), dtype=torch.int32)
    q = torch.randn(T, hq, 128, device=cuda, dtype=torch.bfloat16)
    ctx = torch.tensor(ctx_list, dtype=torch.int32)
    scale = 1 / math.sqrt(128)
    out = torch.empty_like(q)
    ops.prefill_attention(q, kc, vc, bt, cu.to(cuda), ctx.to(cuda), scale, out)
    torch.cuda.synchronize()
    # fp32 reference on up to 96 query rows per sequence (first, last, spread)
    G = hq // hkv
    for i, (ql, cl) in enumerate(cases):
        rows = sorted(set([0, ql - 1] + list(range(0, ql, max(1, ql // 94)))))
        k = ref._gather_kv(kc.cpu(), bt[i].cpu(), cl, bs).float().repeat_interleave(G, dim=1)  # [cl, Hq, D]
        v = ref._gather_kv(vc.cpu(), bt[i].cpu(), cl, bs).float().repeat_interleave(G, dim=1)
        qq = q[cu[i]:cu[i + 1]].cpu().float()
        want = []
        for r in rows:
            c = cl - ql + r + 1  # causal: keys [0, c)
            p = torch.softmax(torch.einsum("hd,khd->hk", qq[r], k[:c]) * scale, -1)
            want.append(torch.einsum("hk,khd->hd", p, v[:c]))
        _close(out[cu[i]:cu[i + 1]][torch.tensor(rows)], torch.stack(want), 0.03, msg=f"prefill long case {i}")


def test_prefill_attention_spike(cuda, pa_variant):
    """Force large online-softmax rescales (guide rule 26): spike one key."""
    hq, hkv, bs = 32, 8, 16
    L = 400
    kc, vc, bt = _paged_setup(cuda, [L], hkv, bs=bs, seed=2)
    q = torch.randn(L, hq, 128, device=cuda, dtype=torch.bfloat16)
    # make key 200 dominate for all queries after it
    blk = bt[0, 200 // bs].item()
    kc[blk, :, 200 % bs] = (q[250, :hkv * 4:4].float() * 8).to(torch.bfloat16)
    cu = torch.tensor([0, L], dtype=torch.int32)
    ctx = torch.tensor([L], dtype=torch.int32)
    out = torch.empty_like(q)
    ops.prefill_attention(q, kc, vc, bt, cu.to(cuda), ctx.to(cuda), 1 / math.sqrt(128), out)
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), cu, ctx, 1 / math.sqrt(128), bs)
    _close(out, exp, 0.03)


def test_rope_cache(cuda):
    hq, hkv, hd, bs = 32, 8, 128, 16
    T = 50
    torch.manual_seed(3)
    qkv = torch.randn(T, (hq + 2 * hkv) * hd, device=cuda, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=cuda)
    cs = ref.rope_cos_sin(hd, 8192, 500000.0, {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                                "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}).to(cuda)
    nb = 8
    kc = torch.zeros(nb, hkv, bs, hd, device=cuda, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    slots = torch.randperm(nb * bs)[:T].to(cuda)
    slots[3] = -1
    kc_r, vc_r, qkv_r = kc.cpu().clone(), vc.cpu().clone(), qkv.cpu().clone()
    ops.rope_cache(qkv, pos, cs, slots, kc, vc, hq, hkv, hd, bs)
    ref.rope_cache(qkv_r, pos.cpu(), cs.cpu(), slots.cpu(), kc_r, vc_r, hq, hkv, hd, bs)
    _close(qkv, qkv_r, 0.03, msg="qkv")
    _close(kc, kc_r, 0.03, msg="k cache")
    _close(vc, vc_r, 0.0, msg="v cache")


def test_silu_and_embedding(cuda):
    gu = torch.randn(33, 2 * 14336, device=cuda, dtype=torch.bfloat16)
    _close(ops.silu_and_mul(gu), ref.silu_and_mul(gu.cpu()), 0.03, 0.01)
    table = torch.randn(1000, 4096, device=cuda, dtype=torch.bfloat16)
    ids = torch.randint(0, 1000, (17,), device=cuda)
    _close(ops.embedding(ids, table), table.cpu()[ids.cpu()], 0.0)
    _close(ops.embedding(ids.int(), table), table.cpu()[ids.cpu()], 0.0)


def test_sample_greedy_and_logprob(cuda):
    torch.manual_seed(4)
    V = 128256
    logits = torch.randn(9, V, device=cuda, dtype=torch.bfloat16) * 3
    t = torch.zeros(9, device=cuda)
    tok, lp = ops.sample(logits, t)
    assert torch.equal(tok.cpu(), logits.float().argmax(-1).cpu())
    exp_lp = torch.log_softmax(logits.float(), -1).gather(1, tok[:, None]).squeeze(1)
    _close(lp, exp_lp, 1e-3)


def test_sample_filters(cuda):
    torch.manual_seed(5)
    V = 50000
    B = 6
    logits = torch.randn(B, V, device=cuda, dtype=torch.float32) * 2
    temp = torch.ones(B, device=cuda)
    topk = torch.tensor([1, 5, 0, 0, 50, 0], dtype=torch.int32, device=cuda)
    topp = torch.tensor([1.0, 1.0, 0.5, 0.9, 0.3, 1.0], device=cuda)
    minp = torch.tensor([0.0, 0.0, 0.0, 0.0, 0.0, 0.2], device=cuda)
    seeds = torch.arange(B, dtype=torch.int64, device=cuda)
    lf = logits.cpu()
    allowed = []
    for i in range(B):
        keep = torch.ones(V, dtype=torch.bool)
        k = int(topk[i])
        if k:
            keep &= lf[i] >= torch.topk(lf[i], k).values[-1]
        if float(minp[i]) > 0:
            keep &= lf[i] >= lf[i].max() + math.log(float(minp[i]))
        p = float(topp[i])
        if p < 1:
            probs = torch.softmax(lf[i].masked_fill(~keep, float("-inf")), -1)
            sp, _ = torch.sort(probs, descending=True)
            n = int((torch.cumsum(sp, 0) < p).sum()) + 1
            keep &= probs >= sp[n - 1] * (1 - 1e-4)
        allowed.append(keep)
    counts = [dict() for _ in range(B)]
    for step in range(64):
        offs = torch.full((B,), step, dtype=torch.int64, device=cuda)
        tok, _ = ops.sample(logits, temp, topk, topp, minp, seeds, offs)
        for i, t in enumerate(tok.tolist()):
            assert allowed[i][t], (i, t)
            counts[i][t] = counts[i].get(t, 0) + 1
    assert len(counts[0]) == 1  # top-k 1 = greedy
    assert len(counts[2]) > 1  # real sampling


def test_sample_distribution(cuda):
    """Exponential race reproduces softmax(x/T) frequencies."""
    V = 8
    x = torch.tensor([[0.0, 1.0, 2.0, 0.5, -1.0, 1.5, 0.2, 3.0]], device=cuda).repeat(4096, 1)
    temp = torch.full((4096,), 1.5, device=cuda)
    seeds = torch.arange(4096, dtype=torch.int64, device=cuda)
    tok, _ = ops.sample(x, temp, None, None, None, seeds, torch.zeros_like(seeds))
    freq = torch.bincount(tok.cpu(), minlength=V).float() / 4096
    exp = torch.softmax(x[0].cpu() / 1.5, -1)
    assert (freq - exp).abs().max() < 0.03


def test_sample_partial_matches_reference_race(cuda):
    """Vocab-sharded sampler half (TP LM head): the kernel's race over a shard
    picks the same global token as the fp32 CPU reference with the same hash
    noise; shard max / sum-exp / logit match; combining two shards equals the
    unsharded result."""
    torch.manual_seed(0)
    B, V = 16, 32064
    logits = (torch.randn(B, V, device=cuda) * 3).to(torch.bfloat16)
    temp = torch.tensor([0.0] * 4 + [0.6, 1.0, 1.5, 0.8] * 3, device=cuda)
    seeds = torch.arange(B, device=cuda) * 7 + 1
    offs = torch.arange(B, device=cuda) % 5
    got = ops.sample_partial(logits, 1000, temp, seeds, offs)
    want = ref.sample_partial(logits.cpu(), 1000, temp.cpu(), seeds.cpu(), offs.cpu())
    g, w = got.cpu(), want
    assert (g[:, 3] == w[:, 3]).float().mean() >= 0.9, (g[:, 3], w[:, 3])  # fast-math log: rare near-ties
    torch.testing.assert_close(g[:, 0], w[:, 0])
    torch.testing.assert_close(g[:, 1], w[:, 1], rtol=1e-3, atol=1e-3)
    same = g[:, 3] == w[:, 3]
    torch.testing.assert_close(g[same, 4], w[same, 4])
    # two shards vs the whole row
    h = V // 2
    parts = torch.stack([ops.sample_partial(logits[:, :h].contiguous(), 0, temp, seeds, offs),
                         ops.sample_partial(logits[:, h:].contiguous(), h, temp, seeds, offs)])
    t2, lp2 = ops.combine_sampled_parts(parts)
    t1, lp1 = ops.combine_sampled_parts(ops.sample_partial(logits, 0, temp, seeds, offs)[None])
    assert torch.equal(t1, t2)
    torch.testing.assert_close(lp1, lp2, rtol=1e-4, atol=1e-4)
    # greedy rows = argmax, logprob = log_softmax at the argmax
    lsm = torch.log_softmax(logits.float(), -1)
    assert torch.equal(t1[:4], logits[:4].float().argmax(-1))
    torch.testing.assert_close(lp1, lsm.gather(1, t1[:, None]).squeeze(1), rtol=1e-3, atol=1e-3)


def test_penalties(cuda):
    V = 100
    logits = torch.randn(2, V, device=cuda)
    outs = [[1, 1, 5], [7]]
    prompts = [[2, 3], [7, 9]]
    exp = ref.apply_penalties(logits.cpu().clone(), outs, prompts, [1.2, 1.0], [0.5, 0.1], [0.3, 0.0])
    ops.apply_penalties(logits, outs, prompts, [1.2, 1.0], [0.5, 0.1], [0.3, 0.0])
    _close(logits, exp, 1e-5)


def test_kv_copy_blocks(cuda):
    L, NB, Hkv, BS, D = 4, 20, 8, 16, 128
    cache = torch.randn(L, 2, NB, Hkv, BS, D, device=cuda, dtype=torch.bfloat16)
    blk_bytes = Hkv * BS * D * 2
    src_ids = torch.tensor([3, 7, 11], dtype=torch.int32, device=cuda)
    # pack all layers/kv of 3 blocks into staging [L*2][3][block]
    stage = torch.empty(L * 2, 3, Hkv, BS, D, device=cuda, dtype=torch.bfloat16)
    dst_ids = torch.arange(3, dtype=torch.int32, device=cuda)
    ops.kv_copy_blocks(stage, cache, src_ids, dst_ids, L * 2, NB * blk_bytes, 3 * blk_bytes, blk_bytes, blk_bytes,
                       blk_bytes)
    torch.cuda.synchronize()
    assert torch.equal(stage.view(L, 2, 3, Hkv, BS, D).cpu(), cache[:, :, [3, 7, 11]].cpu())
    # unpack into other blocks
    cache2 = torch.zeros_like(cache)
    ops.kv_copy_blocks(cache2, stage, dst_ids, torch.tensor([0, 1, 2], dtype=torch.int32, device=cuda), L * 2,
                       3 * blk_bytes, NB * blk_bytes, blk_bytes, blk_bytes, blk_bytes)
    assert torch.equal(cache2[:, :, :3].cpu(), cache[:, :, [3, 7, 11]].cpu())
    # TP relayout: take heads 4..7 of each block (inner offset)
    half = blk_bytes // 2
    stage2 = torch.empty(L * 2, 3, Hkv // 2, BS, D, device=cuda, dtype=torch.bfloat16)
    ops.kv_copy_blocks(stage2, cache, src_ids, dst_ids, L * 2, NB * blk_bytes, 3 * half, blk_bytes, half, half,
                       src_inner_off=half)
    assert torch.equal(stage2.view(L, 2, 3, Hkv // 2, BS, D).cpu(), cache[:, :, [3, 7, 11], 4:].cpu())


def _local_ranks_body(q):
    try:
        from dynamo_exp_amd.parallel.custom_ar import CustomAllReduce

        cuda = torch.device("cuda:0")
        world = 2
        ranks = CustomAllReduce.local_ranks(world, cuda, max_bytes=16 << 20)
        streams = [torch.cuda.Stream() for _ in range(world)]
        errs = []
        for it, rows in enumerate((64, 64, 1024, 64, 1536)):  # one-shot and two-shot (> 1 MiB) interleaved
            xs = [torch.randn(rows, 4096, device=cuda).to(torch.bfloat16) for _ in range(world)]
            want = sum(x.float() for x in xs)
            outs = [torch.empty_like(x) for x in xs]
            torch.cuda.synchronize()
            for r in range(world):
                with torch.cuda.stream(streams[r]):
                    ranks[r].all_reduce(xs[r], out=outs[r], stream=streams[r])
            torch.cuda.synchronize()
            for r in range(world):
                ranks[r].check(blocking=True)
                errs.append((outs[r].float() - want).abs().max().item())
                errs.append(0.0 if torch.equal(outs[r], outs[0]) else 1.0)  # identical on every rank
        for r in ranks:
            r.close()
        q.put(errs)
    except Exception as e:  # noqa: BLE001
        q.put(repr(e))


def test_custom_allreduce_local_ranks(cuda):
    """One-shot all-reduce protocol + kernel with 2 virtual ranks on one GPU,
    each rank's launch on its own stream (they barrier on each other).  Run
    in a fresh process: the two ranks' kernels must sit in different HW
    queues (GPU_MAX_HW_QUEUES, 4 here) to run side by side, and HIP hands a
    process's streams out to its queues in creation order -- after the
    streams earlier tests in this process created, two new streams can land
    on one queue, one rank's kernel then waits behind the other's barrier
    and the barrier times out.  Real ranks are separate processes/GPUs."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_local_ranks_body, args=(q,))
    p.start()
    res = q.get(timeout=100)
    p.join(30)
    assert isinstance(res, list), res
    assert max(res) < 0.06, res


def _failfast_body(q):
    try:
        import time

        from dynamo_exp_amd.parallel.custom_ar import CustomAllReduce

        cuda = torch.device("cuda:0")
        res = {}
        x = torch.ones(64, 4096, device=cuda).to(torch.bfloat16)
        # (a) the flag is already set: 64 all-reduces + 16 all-gathers return at entry
        ranks = CustomAllReduce.local_ranks(2, cuda, max_bytes=1 << 20)
        r0 = ranks[0]
        r0.ep.err.fill_(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(64):
            r0.all_reduce(x)
        for _ in range(16):
            r0.all_gather(x[:8])
        torch.cuda.synchronize()
        res["preset_s"] = time.perf_counter() - t0
        for r in ranks:
            r.close()
        # (b) a peer that never arrives: the first launch times out (0.3 s),
        # the other 63 see the sticky flag and return at once
        ranks = CustomAllReduce.local_ranks(2, cuda, max_bytes=1 << 20)
        r0 = ranks[0]
        r0.timeout_ms = 300
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(64):
            r0.all_reduce(x)
        torch.cuda.synchronize()
        res["timeout_s"] = time.perf_counter() - t0
        res["err"] = int(r0.ep.err.item())
        try:
            r0.check(blocking=True)
            res["raised"] = False
        except RuntimeError:
            res["raised"] = True
        for r in ranks:
            r.close()
        q.put(res)
    except Exception as e:  # noqa: BLE001
        q.put(repr(e))


def test_custom_allreduce_fails_fast_after_a_missed_barrier(cuda):
    """the barrier error flag is sticky and read at kernel
    entry -- with the flag set, 64 all-reduces and 16 all-gathers finish in
    well under a second; with a peer that never arrives, only the FIRST launch
    waits out its timeout and check() raises.  (Round 4: every launch spun its
    own 20 s, so one late rank stalled a captured decode graph for minutes.)"""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_failfast_body, args=(q,))
    p.start()
    res = q.get(timeout=100)
    p.join(30)
    assert isinstance(res, dict), res
    assert res["preset_s"] < 1.0, res
    assert 0.25 < res["timeout_s"] < 1.0, res
    assert res["err"] == 1 and res["raised"], res


def _ar_rank(rank, world, port, q):
    import torch.distributed as dist

    from dynamo_exp_amd.parallel.custom_ar import CustomAllReduce

    os.environ["DX_CUSTOM_AR_SHARED"] = "1"  # both ranks on the one GPU: opt in (custom_ar.py docstring)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
        ar = CustomAllReduce.create(dist.group.WORLD, rank, world, dev, max_bytes=16 << 20)
        errs = []
        for it, rows in enumerate((64, 1024, 8, 1536)):
            g = torch.Generator(device="cpu").manual_seed(1000 * it + rank)
            x = torch.randn(rows, 4096, generator=g).to(torch.bfloat16)
            want = sum(torch.randn(rows, 4096, generator=torch.Generator().manual_seed(1000 * it + r))
                       .to(torch.bfloat16).float() for r in range(world))
            if it % 2:  # producer writes into the registered buffer (no copy)
                buf = ar.buffer((rows, 4096))
                buf.copy_(x.to(dev))
                out = ar.all_reduce(buf)
            else:
                out = ar.all_reduce(x.to(dev))
            torch.cuda.synchronize()
            errs.append((out.float().cpu() - want).abs().max().item())
        # custom all-gather (xGMI peer reads): fp32 sampler partials and bf16 logits shards
        for shape, dt in (((6, 5), torch.float32), ((32, 4000), torch.bfloat16), ((256, 8), torch.float32)):
            mine = torch.full(shape, float(rank + 1), dtype=dt) + torch.arange(shape[-1], dtype=dt)
            got = ar.all_gather(mine.to(dev))
            torch.cuda.synchronize()
            want = torch.stack([torch.full(shape, float(r + 1), dtype=dt) + torch.arange(shape[-1], dtype=dt)
                                for r in range(world)])
            errs.append(0.0 if torch.equal(got.cpu(), want) else 1.0)
        ar.check(blocking=True)
        dist.barrier()
        ar.close()
        dist.barrier()  # every rank dropped its peers' IPC mappings before any producer exits
        q.put((rank, errs))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_custom_allreduce_two_processes_ipc(cuda):
    """CustomAllReduce.create across 2 PROCESSES on one GPU: real IPC-handle
    exchange of the registered buffers and signal arrays (not local_ranks),
    one-shot and two-shot sizes, copy-in and in-place inputs, fp32-summed
    result checked against a CPU sum."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ar_rank, args=(r, 2, 29713, q)) for r in range(2)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=100) for _ in ps)
    [p.join(30) for p in ps]
    for r in range(2):
        assert isinstance(res[r], list), res[r]
        assert max(res[r]) < 0.1, res[r]


@pytest.mark.parametrize("fp8", [False, True])
def test_rope_cache_from_splitk_partials_bit_exact(cuda, fp8):
    """rope_cache on a QKV projection's split-K partials (ops.SplitK) writes the
    same rotated row and the same KV cache bytes as reducing first."""
    Hq, Hkv, D, bs, K = 8, 2, 128, 16, 1024
    N = (Hq + 2 * Hkv) * D
    M = 27
    cfg = (ops.DSTREAM, 4, 1, 2, 4, 2, 4)
    assert ops._dstream_ok(M, N, K, 4, 1, 2, 4, 2, 4)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) * 0.03).to(torch.bfloat16)
    pos = torch.arange(100, 100 + M, device=cuda)
    cos_sin = ref.rope_cos_sin(D, 4096, 500000.0).to(cuda)
    slots = torch.arange(M, device=cuda, dtype=torch.int64) + 5
    slots[3] = -1  # a padded graph slot: no cache write
    dt = ops.KV_FP8 if fp8 else torch.bfloat16
    sc = (0.05, 0.04) if fp8 else (1.0, 1.0)
    caches = [(torch.zeros(8, Hkv, bs, D, device=cuda).to(dt), torch.zeros(8, Hkv, bs, D, device=cuda).to(dt))
              for _ in range(2)]
    y = ops.dstream_linear(x, w, cfg)
    ops.rope_cache(y, pos, cos_sin, slots, caches[0][0], caches[0][1], Hq, Hkv, D, bs, kv_scales=sc)
    p = ops.dstream_linear(x, w, cfg, partial=True)
    out = torch.full_like(y, 7.0)
    got = ops.rope_cache(p, pos, cos_sin, slots, caches[1][0], caches[1][1], Hq, Hkv, D, bs, kv_scales=sc, out=out)
    torch.cuda.synchronize()
    assert got is out and torch.equal(out, y)
    for a, b in zip(caches[0], caches[1]):
        assert torch.equal(a.view(torch.uint8), b.view(torch.uint8))


def test_prefill_attention_bidirectional(cuda):
    """causal=False: every query sees its sequence's whole context (GQA, ragged
    lengths, block 64) -- the vision tower's mode -- vs the fp32 reference."""
    Hq, Hkv, D, bs = 16, 4, 128, 64
    lens = [577, 100, 1030]
    nb = sum(-(-L // bs) for L in lens) + 2
    kc = torch.randn(nb, Hkv, bs, D, device=cuda).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    rows, b = [], 1
    for L in lens:
        n = -(-L // bs)
        rows.append(list(range(b, b + n)) + [0] * (max(-(-x // bs) for x in lens) - n))
        b += n
    bt = torch.tensor(rows, dtype=torch.int32, device=cuda)
    T = sum(lens)
    q = torch.randn(T, Hq, D, device=cuda).to(torch.bfloat16)
    cu = torch.tensor([0] + list(__import__("itertools").accumulate(lens)), dtype=torch.int32, device=cuda)
    ctx = torch.tensor(lens, dtype=torch.int32, device=cuda)
    out = torch.empty_like(q)
    ops.prefill_attention(q, kc, vc, bt, cu, ctx, 0.09, out, causal=False)
    want = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), cu.cpu(), ctx.cpu(), 0.09, bs, causal=False)
    _close(out, want, 0.03, 0.02, "bidirectional prefill attention")
