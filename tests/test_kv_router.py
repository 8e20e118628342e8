"""KV router cost function and routing modes (reference
lib/llm/src/kv_router/scheduler.rs:250-300, examples/llm/components/kv_router.py)."""
import random

from dynamo_exp_amd.llm.kv_router import DefaultWorkerSelector, ForwardPassMetrics, KvRouter


def _m(active, kv_active, kv_total=100):
    return ForwardPassMetrics(request_active_slots=active, request_total_slots=1000, kv_active_blocks=kv_active,
                              kv_total_blocks=kv_total)


def test_load_term_normalised_by_busiest_worker():
    """logit = 2*overlap_score - kv_usage - active/max_active: with the
    reference's normalisation a worker at 10 of 20 active requests pays 0.5,
    not 10/1000 (its own slot count)."""
    sel = DefaultWorkerSelector(block_size=16, rng=random.Random(0))
    ms = {1: _m(20, 10), 2: _m(10, 10)}
    w, logit = sel.select([1, 2], {}, 64, ms)
    assert w == 2 and abs(logit - (0 - 0.1 - 0.5)) < 1e-9
    # one block of overlap (score 16/64 -> +0.5) does not beat a 1.0 load gap
    w, _ = sel.select([1, 2], {1: 1}, 64, {1: _m(20, 10), 2: _m(0, 10)})
    assert w == 2
    # all idle: no division by zero, overlap decides
    w, _ = sel.select([1, 2], {1: 2}, 64, {1: _m(0, 0), 2: _m(0, 0)})
    assert w == 1


class _Comp:
    pass


def test_bumps_apply_to_workers_without_metrics():
    r = KvRouter(_Comp(), 16, selector=DefaultWorkerSelector(16, rng=random.Random(1)))
    r.metrics.update(1, {"request_active_slots": 0, "request_total_slots": 8, "kv_active_blocks": 0,
                         "kv_total_blocks": 100})
    # worker 2 never published: routed requests still count against it
    picks = [r.schedule_sync(list(range(64)), [1, 2])[0] for _ in range(6)]
    assert picks.count(1) == 3 and picks.count(2) == 3


def test_kv_load_mode_picks_least_cache_usage():
    r = KvRouter(_Comp(), 16, selector=DefaultWorkerSelector(16, rng=random.Random(2)))
    assert r.schedule_least_kv_load([1, 2]) == (None, 0.0)  # no metrics: caller falls back to random
    for w, used in ((1, 60), (2, 20), (3, 20)):
        r.metrics.update(w, {"request_active_slots": 1, "request_total_slots": 8, "kv_active_blocks": used,
                             "kv_total_blocks": 100})
    got = {r.schedule_least_kv_load([1, 2, 3])[0] for _ in range(20)}
    assert got == {2, 3}
    assert r.schedule_least_kv_load([1])[0] == 1
