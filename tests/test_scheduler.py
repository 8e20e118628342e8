"""Scheduler policies: chunked prefill with mixed prefill+decode batches vs
the prefill-priority policy (CPU, tiny model)."""
import pytest

from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
from dynamo_exp_amd.engine.request import SamplingParams


def _engine(chunked, budget, model=None, max_seqs=8):
    return LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512, num_gpu_blocks=200,
                                  max_num_seqs=max_seqs, max_num_batched_tokens=budget, chunked_prefill=chunked,
                                  seed=11, async_schedule=False), model=model)  # step-exact batch traces


def _gen(e, prompts, n, trace=None):
    outs = {}
    for i, p in enumerate(prompts):
        e.add_request(f"q{i}", p, SamplingParams(max_tokens=n, ignore_eos=True),
                      on_output=lambda r, t, lp, fin: outs.setdefault(r.request_id, []).extend(t))
    while e.has_unfinished():
        e.step()
        if trace is not None and e.last_batch is not None:
            b = e.last_batch
            trace.append((b.kind, list(b.num_new), list(b.sample), len(b.requests) - b.n_prefill, b.num_tokens))
    return [outs[f"q{i}"] for i in range(len(prompts))]


PROMPTS = [list(range(3 + i, 3 + i + L)) for i, L in enumerate((50, 70, 33, 90))]


def test_chunked_batches_respect_budget_and_mix():
    trace = []
    e = _engine(True, 32)
    outs = _gen(e, PROMPTS, 6, trace)
    assert all(len(o) == 6 for o in outs)
    assert all(t[4] <= 32 for t in trace)
    assert any(k == "mixed" for k, *_ in trace)
    # the first request's 50-token prompt is split 32 + 18
    assert trace[0][:3] == ("prefill", [32], [False])
    assert trace[1][1][0] == 18 and trace[1][2][0] is True
    assert e.stats["mixed_steps"] > 0
    assert not e.scheduler.prefilling and not e.scheduler.running


def test_chunked_matches_unchunked_greedy():
    ref_e = _engine(False, 4096)
    ref = _gen(ref_e, PROMPTS, 8)
    for budget in (24, 64):
        got = _gen(_engine(True, budget, model=ref_e.model), PROMPTS, 8)
        assert got == ref, budget


def test_chunked_with_prefix_cache_and_abort():
    e = _engine(True, 40)
    base = _gen(e, [PROMPTS[3]], 4)[0]
    # same prompt again: 5 cached blocks (80 tokens) are reused; the rest is one chunk
    trace = []
    again = _gen(e, [PROMPTS[3]], 4, trace)[0]
    assert again == base and trace[0][1] == [10]
    # abort a request while its prompt is partially computed
    e.add_request("x", list(range(200, 330)), SamplingParams(max_tokens=4, ignore_eos=True))
    e.step()
    assert e.scheduler.prefilling and e.scheduler.prefilling[0].request_id == "x"
    e.abort("x")
    assert not e.scheduler.prefilling and not e.has_unfinished()
    assert e.kv.num_free() == e.kv.num_blocks


@pytest.mark.parametrize("chunked", [True, False])
def test_preemption_under_kv_pressure(chunked):
    e = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512, num_gpu_blocks=14,
                               max_num_seqs=8, max_num_batched_tokens=64, chunked_prefill=chunked, seed=11))
    outs = _gen(e, [list(range(5, 45)), list(range(50, 90)), list(range(100, 140))], 40)
    assert all(len(o) == 40 for o in outs)
    assert e.scheduler.preemptions > 0


@pytest.mark.parametrize("chunked", [True, False])
def test_preemption_under_kv_pressure_matches_unconstrained(chunked):
    """A pool too small for all streams: growing streams preempt the newest
    ones (recompute), a victim is never scheduled in the same step, and the
    greedy outputs equal an unconstrained run."""
    prompts = [list(range(5 + 7 * i, 5 + 7 * i + 30)) for i in range(6)]
    ref = _gen(_engine(chunked, 4096), prompts, 40)
    e = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512, num_gpu_blocks=14,
                               max_num_seqs=8, max_num_batched_tokens=4096, chunked_prefill=chunked, seed=11))
    got = _gen(e, prompts, 40)
    assert got == ref
    assert e.scheduler.preemptions > 0


def test_prefill_batching_holds_until_tokens_or_delay():
    """min_prefill_tokens / max_prefill_delay: while a stream decodes, a lone
    new prompt waits (decode-only steps) until enough prompt tokens queue or it
    has waited max_prefill_delay; outputs are unchanged."""
    import time

    ref_e = _engine(True, 256)
    ref = _gen(ref_e, PROMPTS, 8)
    e = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512, num_gpu_blocks=200,
                               max_num_seqs=8, max_num_batched_tokens=256, seed=11, min_prefill_tokens=150,
                               max_prefill_delay=30.0), model=ref_e.model)
    outs = {}
    cb = lambda r, t, lp, fin: outs.setdefault(r.request_id, []).extend(t)  # noqa: E731
    e.add_request("q0", PROMPTS[0], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.step()  # nothing decoding yet: no hold
    assert e.last_batch.kind == "prefill"
    e.add_request("q1", PROMPTS[1], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.step()
    assert e.last_batch.kind == "decode"  # 70 queued tokens < 150: held
    e.add_request("q2", PROMPTS[2], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.add_request("q3", PROMPTS[3], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.step()  # 70 + 33 + 90 >= 150: all three prompts in one mixed step
    assert e.last_batch.kind == "mixed" and e.last_batch.n_prefill == 3
    while e.has_unfinished():
        e.step()
    assert [outs[f"q{i}"] for i in range(4)] == ref
    # the delay bound releases a lone prompt
    e.scheduler.cfg.max_prefill_delay = 0.05
    e.add_request("a", PROMPTS[0], SamplingParams(max_tokens=30, ignore_eos=True))
    e.step()
    e.add_request("b", PROMPTS[1], SamplingParams(max_tokens=2, ignore_eos=True))
    e.step()
    assert e.last_batch.n_prefill == 0
    time.sleep(0.06)
    e.step()
    assert e.last_batch.n_prefill == 1


def test_prefill_hold_only_under_load():
    """prefill_hold_min_decode: with fewer decoding streams than the
    threshold a new prompt is not held (light load: TTFT first); once enough
    streams decode, batching holds it again."""
    ref_e = _engine(True, 256)
    e = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512, num_gpu_blocks=200,
                               max_num_seqs=8, max_num_batched_tokens=256, seed=11, min_prefill_tokens=150,
                               max_prefill_delay=30.0, prefill_hold_min_decode=2), model=ref_e.model)
    e.add_request("q0", PROMPTS[0], SamplingParams(max_tokens=20, ignore_eos=True))
    e.step()
    e.add_request("q1", PROMPTS[1], SamplingParams(max_tokens=20, ignore_eos=True))
    e.step()  # one stream decodes (< 2): not held
    assert e.last_batch.n_prefill == 1
    e.add_request("q2", PROMPTS[2], SamplingParams(max_tokens=20, ignore_eos=True))
    e.step()  # two streams decode: held (33 tokens < 150)
    assert e.last_batch.kind == "decode"


def test_prefill_hold_partial_holds_split_remainder():
    """prefill_hold_partial: the remainder of a prompt split by the token
    budget is held with the queue (decode-only steps) until min_prefill_tokens
    are queued or the split request has waited max_prefill_delay; greedy
    outputs are unchanged and a full step follows."""

    ref_e = _engine(True, 64)
    ref = _gen(ref_e, PROMPTS, 8)
    e = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512, num_gpu_blocks=200,
                               max_num_seqs=8, max_num_batched_tokens=64, seed=11, min_prefill_tokens=60,
                               max_prefill_delay=30.0, prefill_hold_partial=1, async_schedule=False),
                  model=ref_e.model)
    outs = {}
    cb = lambda r, t, lp, fin: outs.setdefault(r.request_id, []).extend(t)  # noqa: E731
    e.add_request("q0", PROMPTS[0], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.step()  # nothing decodes yet: 50-token prompt whole
    e.add_request("q1", PROMPTS[1], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.step()  # 70 queued >= 60: mixed step takes 63 of q1's 70 tokens
    assert e.last_batch.kind == "mixed" and e.last_batch.num_new == [63]
    e.step()  # 7-token remainder < 60: held
    assert e.last_batch.kind == "decode"
    e.add_request("q2", PROMPTS[2], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.add_request("q3", PROMPTS[3], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.step()  # 7 + 33 + 90 >= 60: the remainder leads a full step
    b = e.last_batch
    assert b.kind == "mixed" and b.num_new[0] == 7 and b.num_tokens == 64
    while e.has_unfinished():
        e.step()
    assert [outs[f"q{i}"] for i in range(4)] == ref
    # the delay bound releases a held remainder (scheduler clock driven by hand)
    now = [0.0]
    e.scheduler.clock = lambda: now[0]
    e.scheduler.cfg.max_prefill_delay = 0.2
    e.add_request("a", list(range(5, 200)), SamplingParams(max_tokens=40, ignore_eos=True))
    e.step()
    e.step()
    e.add_request("b", list(range(300, 370)), SamplingParams(max_tokens=4, ignore_eos=True))
    while not (e.scheduler.prefilling and e.scheduler.prefilling[0].request_id == "b"):
        e.step()  # "a" finishes its prompt; then "b" is split by the budget
    rb = e.scheduler.prefilling[0]
    rem = len(rb.prompt) - rb.num_computed
    assert 0 < rem < 60
    now[0] = 0.19
    e.step()  # the remainder waits ...
    assert e.last_batch.kind == "decode"
    now[0] = 0.21
    e.step()  # ... until "b" has waited 0.2 s
    assert e.last_batch.n_prefill == 1 and e.last_batch.num_new == [rem]


def test_deferred_whole_prompt_leads_past_the_partial_hold():
    """with prefill_hold_partial AND prefill_whole_prompts on, a
    prompt deferred by the whole-prompt rule leads the next step even when
    the partial hold would fire there (the flag used to be consumed by the
    held step and the deferred prompt held again)."""
    ref_e = _engine(True, 64)
    e = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512, num_gpu_blocks=200,
                               max_num_seqs=8, max_num_batched_tokens=64, seed=11, min_prefill_tokens=60,
                               max_prefill_delay=30.0, prefill_hold_partial=1, prefill_whole_prompts=True,
                               async_schedule=False), model=ref_e.model)
    e.add_request("q0", PROMPTS[0], SamplingParams(max_tokens=8, ignore_eos=True))
    e.step()
    e.add_request("q1", PROMPTS[1], SamplingParams(max_tokens=8, ignore_eos=True))
    e.step()  # q1 split by the budget: 63 of 70
    e.step()  # its 7-token remainder is held (partial hold)
    assert e.last_batch.kind == "decode" and e.scheduler.prefilling
    e.add_request("q2", PROMPTS[2], SamplingParams(max_tokens=8, ignore_eos=True))
    e.step()  # 7 + 33 < 60: still held
    assert e.last_batch.kind == "decode"
    e.scheduler._deferred_whole = True  # as if q2 had been left for this step by the whole-prompt rule
    e.step()
    b = e.last_batch
    assert b.kind == "mixed" and b.num_new == [7, 33], (b.kind, b.num_new)


def test_prefill_whole_prompts_defers_instead_of_splitting():
    """prefill_whole_prompts: once half the budget holds prompt chunks, a new
    prompt that does not fit whole is left for the next step, which it leads
    (past the prefill hold); a prompt larger than the budget is still split;
    greedy outputs are unchanged."""
    ref_e = _engine(True, 128)
    ref = _gen(ref_e, PROMPTS, 8)
    e = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512, num_gpu_blocks=200,
                               max_num_seqs=8, max_num_batched_tokens=128, seed=11, min_prefill_tokens=100,
                               max_prefill_delay=30.0, prefill_whole_prompts=True, async_schedule=False),
                  model=ref_e.model)
    outs = {}
    cb = lambda r, t, lp, fin: outs.setdefault(r.request_id, []).extend(t)  # noqa: E731
    e.add_request("q0", PROMPTS[0], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.step()  # 50 tokens, nothing decoding
    for i in (1, 2, 3):
        e.add_request(f"q{i}", PROMPTS[i], SamplingParams(max_tokens=8, ignore_eos=True), on_output=cb)
    e.step()  # 70 + 33 = 103 >= 64 of the 127 left: q3 (90) does not fit whole -> deferred, not split
    b = e.last_batch
    assert b.kind == "mixed" and b.num_new == [70, 33] and b.sample == [True, True]
    e.step()  # q3 alone (90 < min_prefill_tokens) still goes: it was deferred, not held
    assert e.last_batch.num_new == [90]
    while e.has_unfinished():
        e.step()
    assert [outs[f"q{i}"] for i in range(4)] == ref
    # a prompt larger than the budget is split as before
    e.add_request("big", list(range(7, 307)), SamplingParams(max_tokens=2, ignore_eos=True))
    e.step()
    assert e.last_batch.num_new == [128]
