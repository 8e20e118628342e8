"""Sharded KV indexer and frequency window: the reference's indexer test
cases (lib/llm/src/kv_router/indexer.rs tests: find_matches, early exit,
remove_worker, test_frequency over num_shards {1, 3, 8} x block sizes
{11, 32, 64}) against both the single-tree and the sharded C++ indexers."""
import threading
import time

import pytest

from dynamo_exp_amd.kv import hashing
from dynamo_exp_amd.llm.kv_router import KvIndexer


def _store(idx, worker, hashes, parent=None):
    """reference create_store_event(worker, event_id, hashes, parent): block
    hash == tokens hash == the given ids."""
    idx.apply({"worker_id": worker, "event_id": 0, "stored_parent": parent,
               "stored": [{"block_hash": h, "tokens_hash": h} for h in hashes], "removed": []})


def _remove(idx, worker, hashes):
    idx.apply({"worker_id": worker, "event_id": 0, "stored_parent": None, "stored": [], "removed": list(hashes)})


SHARDS = [1, 3, 8]
BLOCKS = [11, 32, 64]


@pytest.mark.parametrize("shards", SHARDS)
@pytest.mark.parametrize("bs", BLOCKS)
def test_find_matches_empty(shards, bs):
    idx = KvIndexer(bs, shards)
    assert idx.find_matches([hashing.block_hashes(list(b"test data"), 9)[0]]) == {}
    assert idx.find_matches_for_request([1, 2, 3, 4]) == {}


@pytest.mark.parametrize("shards", SHARDS)
def test_overlap_and_remove(shards):
    idx = KvIndexer(16, shards)
    _store(idx, 0, [1, 2, 3])
    _store(idx, 1, [1, 2])
    _store(idx, 2, [7])
    idx.flush()
    assert idx.find_matches([1, 2, 3]) == {0: 3, 1: 2}
    _remove(idx, 0, [3])
    idx.flush()
    assert idx.find_matches([1, 2, 3]) == {0: 2, 1: 2}
    idx.remove_worker(1)
    idx.flush()
    assert idx.find_matches([1, 2, 3]) == {0: 2}
    # a child stored under a parent extends that worker's chain
    _store(idx, 0, [9], parent=2)
    idx.flush()
    assert idx.find_matches([1, 2, 9]) == {0: 3}


def test_early_exit_single_tree():
    """reference test_early_stopping: stop once one worker remains."""
    idx = KvIndexer(16)
    _store(idx, 0, [0, 1, 2])
    _store(idx, 1, [0])
    assert idx.find_matches_scores([0, 1, 2], early_exit=True)[0] == {0: 2, 1: 1}
    assert idx.find_matches_scores([0, 1], early_exit=True)[0] == {0: 2, 1: 1}


def test_workers_spread_over_shards():
    """Least-loaded assignment at a worker's first event (reference
    KvIndexerSharded::apply_event)."""
    idx = KvIndexer(16, 3)
    for w in range(6):
        _store(idx, w, [100 + w])
    idx.flush()
    shard_of = [idx.tree.shard_index(w) for w in range(6)]
    assert sorted(shard_of) == [0, 0, 1, 1, 2, 2]
    assert sorted(idx.tree.workers()) == list(range(6))


@pytest.mark.parametrize("shards", SHARDS)
@pytest.mark.parametrize("bs", BLOCKS)
def test_frequency(shards, bs):
    """reference test_frequency (50 ms window)."""
    idx = KvIndexer(bs, shards, expiration_s=0.05)
    _store(idx, 0, [1, 2, 3, 4])
    idx.flush()
    time.sleep(0.005)
    blocks = [1, 2, 3, 4]
    assert idx.find_matches_scores(blocks)[1] == []
    assert idx.find_matches_scores(blocks)[1] == [1, 1, 1, 1]
    time.sleep(0.1)
    assert idx.find_matches_scores(blocks)[1] == []
    assert idx.find_matches_scores(blocks)[1] == [1, 1, 1, 1]
    assert idx.find_matches_scores(blocks[:3])[1] == [2, 2, 2]
    assert idx.find_matches_scores(blocks)[1] == [3, 3, 3, 2]


def test_sharded_matches_single_tree_under_concurrent_events():
    """Random workload applied from several threads: after a flush the sharded
    indexer answers exactly like the single tree."""
    import random

    rng = random.Random(0)
    single, sharded = KvIndexer(16), KvIndexer(16, 4)
    chains = {w: [] for w in range(12)}
    evs = []
    for _ in range(600):
        w = rng.randrange(12)
        ch = chains[w]
        if ch and rng.random() < 0.3:
            k = rng.randrange(len(ch))
            evs.append(("rm", w, ch[k:]))
            del ch[k:]
        else:
            new = [rng.randrange(1, 50) * 1000 + len(ch) for _ in range(rng.randrange(1, 4))]
            new = [h for h in new if h not in ch][:3]
            if not new:
                continue
            evs.append(("st", w, new, ch[-1] if ch else None))
            ch.extend(new)
    for e in evs:
        if e[0] == "st":
            _store(single, e[1], e[2], e[3])
        else:
            _remove(single, e[1], e[2])
    # per-worker order is all the sharded indexer needs: one thread per worker group
    per = {w: [e for e in evs if e[1] == w] for w in chains}

    def feed(ws):
        for w in ws:
            for e in per[w]:
                if e[0] == "st":
                    _store(sharded, e[1], e[2], e[3])
                else:
                    _remove(sharded, e[1], e[2])

    ts = [threading.Thread(target=feed, args=(list(range(i, 12, 3)),)) for i in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    sharded.flush()
    for w, ch in chains.items():
        if ch:
            assert sharded.find_matches(ch) == single.find_matches(ch)
