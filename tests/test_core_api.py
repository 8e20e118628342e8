"""Reference-named binding API (`dynamo._core` names) over this framework."""
import asyncio

import pytest

from dynamo_exp_amd import _core
from dynamo_exp_amd.kv import hashing
from dynamo_exp_amd.runtime import BackgroundServer


@pytest.fixture(scope="module")
def cp():
    s = BackgroundServer().start()
    yield s.address
    s.stop()


def test_core_api_roundtrip(cp):
    async def main():
        drt = await _core.DistributedRuntime.create(cp)
        etcd = _core.EtcdClient(drt)
        assert etcd.primary_lease_id() != 0
        assert await etcd.kv_create("cfg/x", b"1")
        assert not await etcd.kv_create("cfg/x", b"2")
        cache = await _core.EtcdKvCache.new(etcd, "/dynamo/processor/", {"router": "round-robin"})
        assert await cache.get("router") == b"round-robin"
        await cache.put("router", "kv")
        for _ in range(50):
            if await cache.get("router") == b"kv":
                break
            await asyncio.sleep(0.02)
        assert await cache.get("router") == b"kv"
        comp = drt.namespace("core").component("W")
        idx = _core.KvIndexer(comp, 16)
        agg = _core.KvMetricsAggregator(comp)
        await asyncio.sleep(0.1)
        toks = list(range(32))
        seq, loc = hashing.sequence_hashes(toks, 16), hashing.block_hashes(toks, 16)
        await comp.publish("kv_events", {"worker_id": 5, "event_id": 1, "stored_parent": None, "removed": [],
                                         "stored": [{"block_hash": s, "tokens_hash": h} for s, h in zip(seq, loc)]})
        await comp.publish("load_metrics", {"worker_id": 5, "metrics": {"kv_active_blocks": 3, "kv_total_blocks": 10}})
        await asyncio.sleep(0.2)
        assert idx.find_matches_for_request(toks).scores == {5: 2}
        m = agg.get_metrics().endpoints
        assert m[0]["worker_id"] == 5 and m[0]["kv_active_blocks"] == 3
        assert _core.ModelType.Chat == "chat"
        cache.close()
        await drt.close(1)

    asyncio.run(main())
