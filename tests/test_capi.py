"""C ABI KV-event publisher (reference lib/bindings/c, used by external
engines): events published through libdynamo_llm_capi.so land in the KV
router's indexer with the router's block hashing."""
import asyncio
import ctypes
import os

import pytest

from dynamo_exp_amd.build_native import build_capi
from dynamo_exp_amd.kv import hashing
from dynamo_exp_amd.llm.kv_router import KvIndexer
from dynamo_exp_amd.runtime import BackgroundServer, DistributedRuntime


@pytest.fixture(scope="module")
def lib():
    path = build_capi()
    return ctypes.CDLL(str(path))


def test_capi_publish_into_indexer(lib, monkeypatch):
    srv = BackgroundServer().start()
    monkeypatch.setenv("DX_CONTROL_PLANE", srv.address)
    U64P, SZP, U32P = ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint32)
    lib.dynamo_llm_init.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64, ctypes.c_uint32]
    lib.dynamo_kv_event_publish_stored.argtypes = [ctypes.c_uint64, U32P, SZP, U64P, ctypes.c_size_t, U64P,
                                                   ctypes.c_uint64]
    lib.dynamo_kv_event_publish_removed.argtypes = [ctypes.c_uint64, U64P, ctypes.c_size_t]

    async def main():
        drt = await DistributedRuntime.create(srv.address, is_static=True)
        idx = await KvIndexer(16).start(drt.namespace("capi").component("vllm"))
        await asyncio.sleep(0.1)
        assert lib.dynamo_llm_init(b"capi", b"vllm", 42, 16) == 0
        assert lib.dynamo_llm_init(b"capi", b"vllm", 42, 16) != 0  # one publisher per process
        toks = list(range(1000, 1056))  # 3 full blocks + a partial one (8 tokens)
        seq = hashing.sequence_hashes(toks[:48], 16)
        counts = (ctypes.c_size_t * 4)(16, 16, 16, 8)
        ids = (ctypes.c_uint64 * 4)(*seq, 12345)
        arr = (ctypes.c_uint32 * len(toks))(*toks)

        def pub():
            return lib.dynamo_kv_event_publish_stored(1, arr, counts, ids, 4, None, 0)

        assert await asyncio.to_thread(pub) == 0
        for _ in range(50):
            if idx.events:
                break
            await asyncio.sleep(0.05)
        assert idx.find_matches_for_request(toks) == {42: 3}
        rm = (ctypes.c_uint64 * 1)(seq[2])
        assert await asyncio.to_thread(lib.dynamo_kv_event_publish_removed, 2, rm, 1) == 0
        for _ in range(50):
            if idx.events == 2:
                break
            await asyncio.sleep(0.05)
        assert idx.find_matches_for_request(toks) == {42: 2}
        assert lib.dynamo_llm_shutdown() == 0
        await drt.close(1)

    try:
        asyncio.run(main())
    finally:
        srv.stop()
