"""Native C++ runtime pieces: xxh3, KV hashing (reference test vectors),
radix indexer (mirrors lib/llm/src/kv_router/indexer.rs tests), block pool,
two-part codec (lib/runtime/src/pipeline/network/codec/two_part.rs tests)."""
import random
import struct

import pytest
import xxhash

from dynamo_exp_amd import _native
from dynamo_exp_amd.kv import hashing

R = _native.runtime()
pytestmark = pytest.mark.skipif(R is None, reason="_C_runtime not built")


def test_xxh3_matches_reference_impl():
    rng = random.Random(0)
    for n in list(range(0, 300)) + [511, 512, 1023, 1024, 1025, 2048, 4096, 4097]:
        d = bytes(rng.getrandbits(8) for _ in range(n))
        for seed in (0, 1337, 2**64 - 1):
            assert R.xxh3_64(d, seed) == xxhash.xxh3_64_intdigest(d, seed=seed), (n, seed)


def test_block_hash_vectors_from_reference():
    # lib/llm/src/tokens.rs test_tokens_blocks
    bh, sh = R.block_and_sequence_hashes([1, 2, 3, 4, 5, 6, 7, 8, 9, 10], 4)
    assert bh == [14643705804678351452, 16777012769546811212]
    assert sh == [14643705804678351452, 4945711292740353085]
    assert hashing.sequence_hashes(list(range(1, 11)), 4) == sh


def test_python_fallback_matches(monkeypatch):
    toks = list(range(100, 400))
    native = hashing.block_and_sequence_hashes(toks, 16)
    monkeypatch.setattr(_native, "runtime", lambda: None)
    assert hashing.block_and_sequence_hashes(toks, 16) == native


def _stored(ix, w, parent, hashes):
    return ix.apply_stored(w, parent, hashes, hashes)


def test_radix_store_match_remove():
    ix = R.RadixIndexer()
    _stored(ix, 0, None, [1, 2, 3])
    _stored(ix, 1, None, [1, 2, 4])
    assert ix.find_matches([1, 2, 3]) == {0: 3, 1: 2}
    assert ix.find_matches([1, 2, 4, 5]) == {0: 2, 1: 3}
    assert ix.find_matches([9]) == {}
    # extend worker 0 from parent 3
    _stored(ix, 0, 3, [7])
    assert ix.find_matches([1, 2, 3, 7]) == {0: 4, 1: 2}
    ix.apply_removed(0, [7])
    assert ix.find_matches([1, 2, 3, 7]) == {0: 3, 1: 2}
    ix.remove_worker(1)
    assert ix.find_matches([1, 2, 4]) == {0: 2}
    # pruning: empty leaves disappear
    ix.remove_worker(0)
    assert ix.num_nodes() == 0
    # unknown parent is ignored
    assert _stored(ix, 2, 12345, [1]) == 0


def test_radix_early_exit_and_many_workers():
    ix = R.RadixIndexer()
    for w in range(8):
        _stored(ix, w, None, list(range(w + 1)))
    s = ix.find_matches(list(range(8)))
    assert s == {w: w + 1 for w in range(8)}
    s = ix.find_matches(list(range(8)), True)
    assert max(s.values()) <= 8


def test_block_pool_prefix_and_events():
    p = R.BlockPool(8, True)
    a = p.allocate(3)
    assert len(a) == 3 and p.num_free() == 5
    assert p.register_block(a[0], 111, 11, None)
    assert p.register_block(a[1], 222, 22, 111)
    ev = p.drain_events()
    assert [e[0] for e in ev] == [0, 0] and ev[1][3] == 111
    p.free(a)
    assert p.num_free() == 8 and p.num_cached() == 2
    hit = p.match_prefix([111, 222, 333])
    assert hit == a[:2]
    p.free(hit)
    # exhaust: cached blocks are evicted LRU, emitting removed events
    b = p.allocate(8)
    assert len(b) == 8
    ev = p.drain_events()
    assert sorted(e[1] for e in ev if e[0] == 1) == [111, 222]
    assert p.allocate(1) is None
    with pytest.raises(Exception):
        p.free([b[0], b[0]])


def test_two_part_codec():
    m = R.encode_two_part(b'{"id":1}', b"payload")
    assert len(m) == 24 + 8 + 7
    assert struct.unpack(">QQ", m[:16]) == (8, 7)
    h, b, n = R.decode_two_part(m)
    assert (h, b, n) == (b'{"id":1}', b"payload", len(m))
    assert R.decode_two_part(m[:20]) is None
    assert R.decode_two_part(m[:-1]) is None
    bad = bytearray(m)
    bad[-1] ^= 1
    with pytest.raises(Exception):
        R.decode_two_part(bytes(bad))
    with pytest.raises(Exception):
        R.decode_two_part(m, 10)


def test_event_ring_broadcast_fragments_and_close():
    """csrc/runtime/event_ring.h: every consumer sees every message in order,
    messages larger than a slot are fragmented/reassembled, a slow consumer
    back-pressures the producer (4 slots, 40 messages), close ends polls."""
    import os
    import threading

    from dynamo_exp_amd import _native

    rt = _native.runtime()
    name = f"/dx_test_ring_{os.getpid()}"
    prod = rt.EventRing.create(name, 4, 64, 2)
    cons = [rt.EventRing.attach(name, i) for i in range(2)]
    prod.unlink()  # mapped by everyone already
    msgs = [os.urandom(n) for n in (0, 10, 64, 65, 300)] * 8
    got = {0: [], 1: []}

    def run(c, i):
        for _ in msgs:
            got[i].append(c.poll(10.0))

    ts = [threading.Thread(target=run, args=(c, i)) for i, c in enumerate(cons)]
    [t.start() for t in ts]
    for m in msgs:
        assert prod.publish(m, 10.0)
    [t.join() for t in ts]
    assert got[0] == msgs and got[1] == msgs
    assert cons[0].poll(0.01) is None  # nothing pending: timeout
    prod.close()
    assert cons[1].poll(0.01) is None and cons[1].closed
