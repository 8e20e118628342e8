"""Pinned-host KV tier: blocks evicted from the device pool are demoted to
host memory and promoted back on a later prefix hit (reference KV block
manager v2 host storage, docs/kv_cache_manager.md)."""
import pytest
import torch

from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
from dynamo_exp_amd.engine.request import SamplingParams


def _run(e, rid, prompt, n=6):
    out = []
    e.add_request(rid, prompt, SamplingParams(max_tokens=n, ignore_eos=True), on_output=lambda r, t, lp, f: out.extend(t))
    while e.has_unfinished():
        e.step()
    return out


def _engine(device, host_blocks, model=None):
    return LLMEngine(EngineConfig(model="tiny", device=device, block_size=16, max_model_len=256, num_gpu_blocks=16,
                                  max_num_seqs=4, host_kv_blocks=host_blocks, seed=7, use_cuda_graph=False),
                     model=model)


def _check(device):
    e = _engine(device, 64)
    A = list(range(100, 196))  # 6 blocks
    ref = _run(e, "a", A)
    # push A's cached blocks out of the 16-block device pool
    for i in range(3):
        _run(e, f"x{i}", list(range(200 + 97 * i, 200 + 97 * i + 96)))
    st = e.host_tier.stats
    assert st["demoted"] + st["written_ahead"] >= 5
    got = _run(e, "a2", A)
    assert got == ref
    assert e.kv.host_hit_tokens >= 5 * 16
    assert e.host_tier.stats["promoted"] >= 5
    # without a host tier the same sequence recomputes everything
    e2 = _engine(device, 0, model=e.model)
    _run(e2, "a", A)
    for i in range(3):
        _run(e2, f"x{i}", list(range(200 + 97 * i, 200 + 97 * i + 96)))
    assert _run(e2, "a2", A) == ref and e2.kv.host_hit_tokens == 0


def test_host_tier_cpu():
    _check("cpu")


@pytest.mark.gpu
def test_host_tier_gpu(cuda):
    _check("cuda:0")


def test_multiturn_bench_host_tier_reuse():
    """tools/multiturn_bench.py on the CPU engine: with a device pool smaller than
    the users' histories, GPU-only prefix caching loses the prefixes between rounds
    while the host tier serves them back (promotions, host-hit tokens > 0)."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import multiturn_bench

    off, on = multiturn_bench.main(["--cpu", "--model", "tiny", "--users", "4", "--rounds", "3", "--first", "128",
                                    "--turn", "16", "--osl", "8", "--block-size", "16", "--gpu-blocks", "24",
                                    "--host-blocks", "0,64"])
    assert all(r["host_hit_tokens"] == 0 for r in off["rounds"])
    assert sum(r["prefix_hit_tokens"] for r in on["rounds"][1:]) > sum(r["prefix_hit_tokens"] for r in off["rounds"][1:])
    assert on["rounds"][1]["host_hit_tokens"] > 0 and on["host_tier"]["promoted"] > 0


def test_priority_eviction_order():
    """Released cached blocks are evicted lowest priority first, then oldest
    release (reference kv/reuse.rs PriorityKey)."""
    from dynamo_exp_amd import _native

    p = _native.runtime().BlockPool(4, True)
    ids = p.allocate(4)
    for i, b in enumerate(ids):
        p.register_block(b, 1000 + i, 2000 + i, None)
    p.free([ids[0]], priority=5)  # oldest, but high priority
    p.free([ids[1]])  # priority 0
    p.free([ids[2]])
    p.free([ids[3]], priority=1)
    assert p.lru_candidates(4) == [ids[1], ids[2], ids[3], ids[0]]
    assert p.set_priority(1001, 9)  # reference update_block re-ranks a cached block
    assert p.lru_candidates(4) == [ids[2], ids[3], ids[0], ids[1]]
    got = p.allocate(2)  # evicts the two lowest-ranked
    assert sorted(got) == sorted([ids[2], ids[3]])
    assert p.count_prefix([1000]) == 1 and p.count_prefix([1001]) == 1 and p.count_prefix([1002]) == 0


def test_router_sees_host_tier_blocks():
    """Host-resident prefixes keep counting as the worker's overlap: the KV
    manager merges both tiers' events, so a demotion is not a Removed event
    and a host eviction (nothing left on either tier) is."""
    from dynamo_exp_amd.kv import hashing
    from dynamo_exp_amd.llm.kv_router import KvEventPublisher, KvIndexer

    e = _engine("cpu", 24)
    idx = KvIndexer(16)
    pub = KvEventPublisher(None, 7, 16)
    e.add_kv_event_listener(lambda evs: idx.apply(pub.make_event(evs)))
    A = list(range(100, 196))  # 6 full blocks
    _run(e, "a", A)
    _, sh = hashing.block_and_sequence_hashes(A, 16)
    assert idx.find_matches_for_request(A).get(7, 0) >= 5
    for i in range(3):  # A leaves the device pool (16 blocks) ...
        _run(e, f"x{i}", list(range(200 + 97 * i, 200 + 97 * i + 96)))
    assert e.kv.pool.count_prefix(sh) < 5 <= e.host_tier.count(sh)
    assert idx.find_matches_for_request(A).get(7, 0) >= 5  # ... but the router still counts it (host tier)
    for i in range(3, 20):  # the 24-block host tier overflows: A's blocks leave both tiers
        _run(e, f"x{i}", list(range(20 * i, 20 * i + 96)))
        if e.host_tier.count(sh) == 0:
            break
    assert e.host_tier.count(sh) == 0
    assert idx.find_matches_for_request(A).get(7, 0) == e.kv.pool.count_prefix(sh)


def test_auto_host_blocks():
    from dynamo_exp_amd.engine.host_tier import auto_host_blocks

    n = auto_host_blocks(1 << 20, 1000)
    assert 0 < n <= 4000
    assert auto_host_blocks(1 << 60, 1000) == 0  # nothing fits
