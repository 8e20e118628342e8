"""Distributed runtime over the real in-tree control plane (spawned in-process,
like the reference's pytest fixtures spawn nats-server + etcd)."""
import asyncio

import pytest

from dynamo_exp_amd.runtime import BackgroundServer, Context, DistributedRuntime, EndpointError
from dynamo_exp_amd.runtime.control_plane import ControlPlaneClient, subject_matches


@pytest.fixture(scope="module", params=["python", "native"])
def cp(request):
    """Every runtime test runs against both control-plane servers: the asyncio
    one and the native dx-ctrld (csrc/ctrld), which speak the same protocol."""
    if request.param == "native":
        from dynamo_exp_amd.build_native import build_ctrld
        from dynamo_exp_amd.runtime.control_plane import NativeServerProcess

        build_ctrld()
        s = NativeServerProcess("127.0.0.1", 0).start()
    else:
        s = BackgroundServer().start()
    yield s.address
    s.stop()


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


def test_subject_matching():
    assert subject_matches("a.b.c", "a.b.c")
    assert subject_matches("a.*.c", "a.x.c")
    assert not subject_matches("a.*.c", "a.x.d")
    assert subject_matches("a.>", "a.x.y.z")
    assert not subject_matches("a.>", "a")
    assert not subject_matches("a.b", "a.b.c")


def test_kv_leases_watch(cp):
    async def main():
        c = await ControlPlaneClient(cp).connect()
        await c.put("t1/a", b"1")
        assert await c.get("t1/a") == b"1"
        assert not await c.create("t1/a", b"2")
        assert await c.create("t1/b", b"2")
        assert await c.create_or_validate("t1/b", b"2")
        assert not await c.create_or_validate("t1/b", b"3")
        st = await c.watch_prefix("t1/")
        snap = await st.__anext__()
        assert [k for k, _, _ in snap["items"]] == ["t1/a", "t1/b"]
        lease = await c.lease_grant(0.3)
        await c.put("t1/leased", b"x", lease=lease)
        ev = await st.__anext__()
        assert ev["type"] == "put" and ev["key"] == "t1/leased"
        # no keepalive -> expiry deletes the key
        ev = await asyncio.wait_for(st.__anext__(), 3)
        assert ev["type"] == "delete" and ev["key"] == "t1/leased"
        lease2 = await c.lease_grant(5)
        await c.put("t1/l2", b"y", lease=lease2)
        await st.__anext__()
        assert await c.lease_revoke(lease2) == 1
        assert (await st.__anext__())["type"] == "delete"
        await st.cancel()
        await c.close()

    run(main())


def test_pubsub_queue_blob(cp):
    async def main():
        c = await ControlPlaneClient(cp).connect()
        sub = await c.subscribe("ev.*.x")
        await c.publish("ev.1.x", b"hello")
        await c.publish("ev.1.y", b"nope")
        item = await asyncio.wait_for(sub.__anext__(), 2)
        assert item["data"] == b"hello"
        await sub.cancel()
        # work queue with ack / redelivery
        await c.q_push("pq", b"m1")
        await c.q_push("pq", b"m2")
        assert await c.q_size("pq") == 2
        m = await c.q_pop("pq", timeout=1, ack_wait=0.2)
        assert m["data"] == b"m1"
        await asyncio.sleep(0.5)  # not acked -> redelivered first
        m = await c.q_pop("pq", timeout=1)
        assert m["data"] == b"m1" and m["deliveries"] == 2
        assert await c.q_ack("pq", m["seq"])
        m = await c.q_pop("pq", timeout=1)
        assert m["data"] == b"m2"
        await c.q_ack("pq", m["seq"])
        assert await c.q_pop("pq", timeout=0.1) is None
        # blocking pop woken by a push
        waiter = asyncio.create_task(c.q_pop("pq", timeout=3))
        await asyncio.sleep(0.1)
        await c.q_push("pq", b"late")
        assert (await waiter)["data"] == b"late"
        await c.blob_put("mdc", "tokenizer.json", b"{}")
        assert await c.blob_get("mdc", "tokenizer.json") == b"{}"
        assert await c.blob_list("mdc") == ["tokenizer.json"]
        await c.close()

    run(main())


def test_endpoint_stream_discovery_and_cancel(cp):
    async def main():
        server = await DistributedRuntime.create(cp)
        client_rt = await DistributedRuntime.create(cp)
        ep = server.namespace("test").component("echo").endpoint("generate")
        stopped = asyncio.Event()

        async def handler(req, ctx: Context):
            for i in range(req["n"]):
                if ctx.is_stopped():
                    stopped.set()
                    return
                yield {"i": i, "text": req["text"]}
                await asyncio.sleep(0.01)

        async def failing(req):
            raise ValueError("bad request")
            yield  # noqa

        await ep.register(handler, stats_handler=lambda: {"load": 0.5})
        await server.namespace("test").component("echo").endpoint("fail").register(failing)
        cl = await client_rt.namespace("test").component("echo").endpoint("generate").client()
        ids = await cl.wait_for_instances(timeout=5)
        assert ids == [server.primary_lease.id]
        out = [x async for x in await cl.round_robin({"n": 3, "text": "hi"})]
        assert [o["i"] for o in out] == [0, 1, 2]
        out = [x async for x in await cl.direct({"n": 2, "text": "d"}, ids[0])]
        assert len(out) == 2
        # graceful stop from the caller
        ctx = Context()
        stream = await cl.random({"n": 1000, "text": "x"}, ctx)
        got = 0
        async for _ in stream:
            got += 1
            if got == 3:
                ctx.stop_generating()
        await asyncio.wait_for(stopped.wait(), 5)
        assert got < 1000
        # errors travel in the stream
        fcl = await client_rt.namespace("test").component("echo").endpoint("fail").client()
        await fcl.wait_for_instances(timeout=5)
        with pytest.raises(EndpointError):
            async for _ in await fcl.generate({}):
                pass
        stats = await client_rt.namespace("test").component("echo").scrape_stats()
        assert any(s["data"] == {"load": 0.5} for s in stats)
        # lease revoke removes the instance from discovery
        await server.primary_lease.revoke()
        for _ in range(100):
            if not cl.instance_ids():
                break
            await asyncio.sleep(0.02)
        assert cl.instance_ids() == []
        await cl.close()
        await fcl.close()
        await server.close(1)
        await client_rt.close(1)

    run(main())


def test_events(cp):
    async def main():
        rt = await DistributedRuntime.create(cp)
        comp = rt.namespace("ev").component("w")
        sub = await comp.subscribe("kv_events")
        await comp.publish("kv_events", {"a": 1})
        got = await asyncio.wait_for(sub.__anext__(), 2)
        assert got == {"a": 1}
        await rt.close(1)

    run(main())


def test_runtime_config_layering(tmp_path, monkeypatch):
    from dynamo_exp_amd.runtime.config import RuntimeConfig, WorkerConfig, is_truthy

    base = tmp_path / "defaults.toml"
    base.write_text("num_worker_threads = 4\nmax_blocking_threads = 8\n")
    over = tmp_path / "etc.toml"
    over.write_text("max_blocking_threads = 32\n")
    cfg = RuntimeConfig.from_settings(files=(str(base), str(over)), env={})
    assert (cfg.num_worker_threads, cfg.max_blocking_threads) == (4, 32)
    cfg = RuntimeConfig.from_settings(files=(str(base), str(over)),
                                      env={"DYN_RUNTIME_NUM_WORKER_THREADS": "2", "DYN_RUNTIME_MAX_BLOCKING_THREADS": ""})
    assert (cfg.num_worker_threads, cfg.max_blocking_threads) == (2, 32)
    with pytest.raises(ValueError):
        RuntimeConfig.from_settings(files=(), env={"DYN_RUNTIME_NUM_WORKER_THREADS": "0"})
    assert WorkerConfig.from_settings({"DYN_WORKER_GRACEFUL_SHUTDOWN_TIMEOUT": "3"}).graceful_shutdown_timeout == 3
    assert is_truthy("On") and is_truthy("1") and not is_truthy("0") and not is_truthy(None)


def test_corrupt_frame_closes_connection_cleanly(cp):
    """A frame whose checksum does not match (N1 two-part codec) ends that one
    connection with a logged error; the endpoint server keeps serving."""
    import struct

    async def main():
        server = await DistributedRuntime.create(cp)
        client_rt = await DistributedRuntime.create(cp)
        ep = server.namespace("t").component("c").endpoint("gen")

        async def handler(req):
            yield {"ok": req["x"]}

        await ep.register(handler)
        host, port = server.server.address.rsplit(":", 1)
        r, w = await asyncio.open_connection(host, int(port))
        w.write(struct.pack(">QQQ", 2, 3, 12345) + b"{}" + b"abc")  # wrong checksum
        await w.drain()
        assert await asyncio.wait_for(r.read(), 5) == b""  # server closed it
        w.close()
        cl = await client_rt.namespace("t").component("c").endpoint("gen").client()
        await cl.wait_for_instances(timeout=5)
        out = [x async for x in await cl.round_robin({"x": 7})]
        assert out == [{"ok": 7}]
        await cl.close()
        await server.close(1)
        await client_rt.close(1)

    run(main())


def test_soak_batches_of_concurrent_streams(cp):
    """Soak (reference lib/runtime/tests/soak.rs): batches of concurrent streaming requests through discovery ->
    random routing -> the endpoint's TCP response stream, repeated until a time budget is spent, every stream
    complete and in order.  Two server runtimes serve the endpoint; both must take traffic.  CI sizes it small;
    DX_SOAK_BATCH / DX_SOAK_SECONDS scale it up (reference defaults: 10000 per batch, 1 minute)."""
    import os
    import time

    batch = int(os.environ.get("DX_SOAK_BATCH", "300"))
    seconds = float(os.environ.get("DX_SOAK_SECONDS", "2"))
    text = "hello world"

    async def main():
        servers = [await DistributedRuntime.create(cp) for _ in range(2)]
        client_rt = await DistributedRuntime.create(cp)
        served = {}
        for i, rt in enumerate(servers):
            async def handler(req, ctx, i=i):
                served[i] = served.get(i, 0) + 1
                for ch in req:
                    yield ch
                    await asyncio.sleep(0.001)

            await rt.namespace("soak").component("backend").endpoint("generate").register(handler)
        cl = await client_rt.namespace("soak").component("backend").endpoint("generate").client()
        for _ in range(200):
            if len(cl.instance_ids()) == 2:
                break
            await asyncio.sleep(0.02)
        assert len(cl.instance_ids()) == 2

        async def one():
            stream = await asyncio.wait_for(cl.random(text), 30)
            out = []
            async for ch in stream:
                out.append(ch)
            return "".join(out)

        t0, count = time.monotonic(), 0
        while True:
            got = await asyncio.gather(*(one() for _ in range(batch)))
            assert got == [text] * batch
            count += batch
            if time.monotonic() - t0 > seconds:
                break
        assert count >= batch and sum(served.values()) == count
        assert all(served.get(i, 0) > 0 for i in range(2)), served
        await cl.close()
        for rt in servers:
            await rt.close(1)
        await client_rt.close(1)

    asyncio.run(asyncio.wait_for(main(), 120))
