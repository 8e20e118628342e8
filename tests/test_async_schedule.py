"""Asynchronous scheduling (EngineConfig.async_schedule): step t+1 is
scheduled and enqueued before step t's tokens are read back, its decode
inputs patched from the device.  Token streams must equal the synchronous
engine's exactly (greedy), across prompt chunking, EOS stops inside the
lookahead, aborts, preemption and prefill-first batches."""
import random

import pytest

from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
from dynamo_exp_amd.engine.request import SamplingParams


def _engine(async_schedule, chunked=True, blocks=400, model=None, budget=96):
    return LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512,
                                  num_gpu_blocks=blocks, max_num_seqs=6, max_num_batched_tokens=budget,
                                  chunked_prefill=chunked, seed=3, async_schedule=async_schedule), model=model)


def _run(eng, reqs, arrivals=None, abort_at=None):
    outs, fins = {}, {}
    arrivals = arrivals or {}
    pending = list(reqs)
    it = 0
    while pending or eng.has_unfinished():
        for rid, prompt, params in [p for p in pending if arrivals.get(p[0], 0) <= it]:
            eng.add_request(rid, prompt, params,
                            on_output=lambda r, t, lp, f: (outs.setdefault(r.request_id, []).extend(t),
                                                           f and fins.setdefault(r.request_id, r.finish_reason)))
            pending = [p for p in pending if p[0] != rid]
        if abort_at and it == abort_at[1]:
            eng.abort(abort_at[0])
        eng.step()
        it += 1
        assert it < 5000
    return outs, fins


def _workload(seed, eos=None):
    rng = random.Random(seed)
    reqs = []
    for i in range(9):
        n = rng.randint(20, 140)
        prompt = [rng.randrange(3, 500) for _ in range(n)]
        sp = SamplingParams(max_tokens=rng.randint(1, 24), ignore_eos=eos is None,
                            stop_token_ids=[] if eos is None else [eos])
        reqs.append((f"r{i}", prompt, sp))
    arrivals = {f"r{i}": rng.randint(0, 12) for i in range(9)}
    return reqs, arrivals


@pytest.mark.parametrize("chunked", [True, False])
def test_async_matches_sync(chunked):
    sync_e = _engine(False, chunked)
    async_e = _engine(True, chunked, model=sync_e.model)
    reqs, arr = _workload(1)
    a = _run(sync_e, [(r, p, SamplingParams(**vars(s))) for r, p, s in reqs], arr)
    b = _run(async_e, [(r, p, SamplingParams(**vars(s))) for r, p, s in reqs], arr)
    assert a == b
    assert all(len(v) == s.max_tokens for (r, _, s), v in zip(reqs, [a[0][r] for r, _, _ in reqs]))


def test_async_stops_inside_lookahead():
    """An EOS sampled at step t while step t+1 (with that request) is already
    enqueued: the stale token is dropped, outputs equal the synchronous run."""
    sync_e = _engine(False)
    async_e = _engine(True, model=sync_e.model)
    # pick an eos that the tiny model actually emits: the 3rd token of a probe run
    probe = _run(_engine(False, model=sync_e.model), [("p", list(range(40, 90)), SamplingParams(max_tokens=8,
                                                                                                 ignore_eos=True))])
    eos = probe[0]["p"][2]
    reqs, arr = _workload(2, eos=eos)
    reqs.append(("probe", list(range(40, 90)), SamplingParams(max_tokens=8, stop_token_ids=[eos])))
    a = _run(sync_e, [(r, p, SamplingParams(**vars(s))) for r, p, s in reqs], arr)
    b = _run(async_e, [(r, p, SamplingParams(**vars(s))) for r, p, s in reqs], arr)
    assert a == b
    assert a[0]["probe"] == probe[0]["p"][:3] and a[1]["probe"].value == "stop"


def test_async_abort_and_preemption():
    """Tight KV pool (preemption) and an abort while a token is in flight."""
    sync_e = _engine(False, blocks=24)
    async_e = _engine(True, blocks=24, model=sync_e.model)
    reqs, arr = _workload(3)
    a = _run(sync_e, [(r, p, SamplingParams(**vars(s))) for r, p, s in reqs], arr, abort_at=("r2", 6))
    b = _run(async_e, [(r, p, SamplingParams(**vars(s))) for r, p, s in reqs], arr, abort_at=("r2", 6))
    assert async_e.scheduler.preemptions > 0
    done_a = {k: v for k, v in a[0].items() if k != "r2"}
    done_b = {k: v for k, v in b[0].items() if k != "r2"}
    assert done_a == done_b
    assert b[1]["r2"].value == "cancelled"
    assert not async_e.has_unfinished() and async_e.kv.num_free() == 24
