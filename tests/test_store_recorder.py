"""Key-value store backends + JSONL recorder / KV-event replay (reference
key_value_store/mem.rs tests, recorder.rs tests, test_kv_bindings replay)."""
import asyncio
import os

import pytest

from dynamo_exp_amd.kv import hashing
from dynamo_exp_amd.llm.kv_router import KvIndexer
from dynamo_exp_amd.llm.kv_store import ControlPlaneStorage, KeyValueStoreManager, MemoryStorage
from dynamo_exp_amd.llm.recorder import KvRecorder, Recorder, read_events, replay_events
from dynamo_exp_amd.runtime import BackgroundServer, DistributedRuntime


@pytest.fixture(scope="module")
def cp():
    s = BackgroundServer().start()
    yield s.address
    s.stop()


async def _store_semantics(store):
    m = KeyValueStoreManager(store)
    obj = {"name": "card", "revision": 0}
    assert (await m.publish("cards", "k1", obj)).kind == "created"
    assert (await m.publish("cards", "k1", obj)).kind == "exists"
    obj["revision"] = 5
    obj["name"] = "card2"
    assert (await m.publish("cards", "k1", obj)).kind == "created"
    assert (await m.load("cards", "k1"))["name"] == "card2"
    assert await m.load("nobucket", "k1") is None
    seen = []

    async def watch():
        async for o in m.watch("cards"):
            seen.append(o["name"])
            if len(seen) == 2:
                return

    t = asyncio.create_task(watch())
    await asyncio.sleep(0.1)
    await m.publish("cards", "k2", {"name": "other", "revision": 1})
    await asyncio.wait_for(t, 5)
    assert seen == ["card2", "other"]
    b = await store.get_bucket("cards")
    await b.delete("k1")
    assert set(await b.entries()) == {"k2"}


def test_memory_store():
    asyncio.run(_store_semantics(MemoryStorage()))


def test_control_plane_store(cp):
    async def main():
        drt = await DistributedRuntime.create(cp, is_static=True)
        await _store_semantics(ControlPlaneStorage(drt.cp))
        # TTL bucket: items vanish unless re-published
        st = ControlPlaneStorage(drt.cp)
        b = await st.get_or_create_bucket("ttl", ttl=0.5)
        await b.insert("x", "v", 1)
        assert await b.get("x") == b"v"
        for _ in range(40):
            await asyncio.sleep(0.1)
            if await b.get("x") is None:
                break
        assert await b.get("x") is None
        await drt.close(1)

    asyncio.run(main())


def test_recorder_rotation_and_limits(tmp_path):
    p = str(tmp_path / "ev.jsonl")
    r = Recorder(p, max_lines_per_file=3, max_count=7)
    for i in range(10):
        r.record({"i": i})
    r.close()
    assert r.count == 7 and len(r.files()) == 3 and all(os.path.exists(f) for f in r.files())
    evs = list(read_events(p))
    assert [e["i"] for _, e in evs] == list(range(7))
    assert all(evs[i][0] <= evs[i + 1][0] for i in range(6))


def test_kv_recorder_replay(cp, tmp_path):
    async def main():
        drt = await DistributedRuntime.create(cp, is_static=True)
        comp = drt.namespace("rec").component("W")
        path = str(tmp_path / "kv.jsonl")
        rec = await KvRecorder(comp, path).start()
        toks = list(range(64))
        seq, loc = hashing.sequence_hashes(toks, 16), hashing.block_hashes(toks, 16)
        await asyncio.sleep(0.1)
        await comp.publish("kv_events", {"worker_id": 7, "event_id": 1, "stored_parent": None,
                                         "stored": [{"block_hash": s, "tokens_hash": h} for s, h in zip(seq, loc)],
                                         "removed": []})
        await comp.publish("kv_events", {"worker_id": 7, "event_id": 2, "stored_parent": None, "stored": [],
                                         "removed": [seq[-1]]})
        for _ in range(50):
            if rec.event_count == 2:
                break
            await asyncio.sleep(0.05)
        rec.shutdown()
        idx = KvIndexer(16)
        assert await replay_events(path, idx, timed=True, speedup=100) == 2
        assert idx.find_matches_for_request(toks) == {7: 3}
        await drt.close(1)

    asyncio.run(main())
