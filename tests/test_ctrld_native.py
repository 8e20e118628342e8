"""Native control-plane server (csrc/ctrld -> bin/dx-ctrld).

* differential test: a random sequence of KV / lease / queue / blob operations
  returns identical results from the native server and the asyncio
  ControlPlaneServer (lease ids, times and server-identity fields masked);
* watch ordering under concurrent writers; pop-waiter cancellation;
* a malformed frame drops that connection only.
"""
import asyncio
import random
import socket
import struct

import pytest

from dynamo_exp_amd.runtime import BackgroundServer
from dynamo_exp_amd.runtime.control_plane import ControlPlaneClient, NativeServerProcess


@pytest.fixture(scope="module")
def native():
    from dynamo_exp_amd.build_native import build_ctrld

    build_ctrld()
    s = NativeServerProcess("127.0.0.1", 0).start()
    yield s.address
    s.stop()


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 60))


async def _script(addr: str, seed: int) -> list:
    rng = random.Random(seed)
    c = await ControlPlaneClient(addr).connect()
    out = []
    leases = []
    keys = [f"d{seed}/k{i}" for i in range(12)] + [f"d{seed}/sub/k{i}" for i in range(6)]
    for step in range(400):
        op = rng.choice(["put", "get", "create", "cov", "del", "prefix", "delp", "lease", "revoke", "lput",
                         "push", "pop", "ack", "nak", "size", "blob", "bget", "blist", "bdel"])
        k = rng.choice(keys)
        v = bytes([rng.randrange(256) for _ in range(rng.randrange(0, 40))])
        q = f"q{seed}_{rng.randrange(2)}"
        if op == "put":
            out.append(("put", await c.call("put", key=k, value=v)))
        elif op == "get":
            r = await c.call("get", key=k)
            if r is not None:
                r = {**r, "lease": r["lease"] is not None}
            out.append(("get", r))
        elif op == "create":
            out.append(("create", await c.call("create", key=k, value=v)))
        elif op == "cov":
            out.append(("cov", await c.call("create_or_validate", key=k, value=v[:1])))
        elif op == "del":
            out.append(("del", await c.call("delete", key=k)))
        elif op == "prefix":
            out.append(("prefix", await c.call("get_prefix", prefix=f"d{seed}/sub/")))
        elif op == "delp":
            if rng.random() < 0.2:
                out.append(("delp", await c.call("delete_prefix", prefix=f"d{seed}/sub/")))
        elif op == "lease":
            r = await c.call("lease_grant", ttl=100.0)
            leases.append(r["lease"])
            out.append(("lease", r["ttl"]))
        elif op == "revoke" and leases:
            lid = leases.pop(rng.randrange(len(leases)))
            out.append(("revoke", await c.call("lease_revoke", lease=lid)))
        elif op == "lput" and leases:
            out.append(("lput", await c.call("put", key=k, value=v, lease=rng.choice(leases))))
        elif op == "push":
            out.append(("push", await c.call("q_push", queue=q, data=v)))
        elif op == "pop":
            out.append(("pop", await c.call("q_pop", queue=q, timeout=0.0, ack_wait=100.0)))
        elif op == "ack":
            out.append(("ack", await c.call("q_ack", queue=q, seq=rng.randrange(1, 30))))
        elif op == "nak":
            out.append(("nak", await c.call("q_nak", queue=q, seq=rng.randrange(1, 30))))
        elif op == "size":
            out.append(("size", await c.call("q_size", queue=q)))
        elif op == "blob":
            out.append(("blob", await c.call("blob_put", bucket="b", key=k, data=v, ttl=None)))
        elif op == "bget":
            out.append(("bget", await c.call("blob_get", bucket="b", key=k)))
        elif op == "blist":
            out.append(("blist", await c.call("blob_list", bucket="b")))
        elif op == "bdel":
            out.append(("bdel", await c.call("blob_delete", bucket="b", key=k)))
    await c.close()
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_native_matches_asyncio_server(native, seed):
    py = BackgroundServer().start()
    nat = NativeServerProcess("127.0.0.1", 0).start()  # fresh: revisions start at 0 on both
    try:
        ref = run(_script(py.address, seed))
        got = run(_script(nat.address, seed))
    finally:
        py.stop()
        nat.stop()
    assert len(got) == len(ref)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert a == b, (i, a, b)


def test_watch_sees_every_write_in_revision_order(native):
    async def main():
        watcher = await ControlPlaneClient(native).connect()
        st = await watcher.watch_prefix("wo/")
        snap = await st.__anext__()
        assert snap["type"] == "snapshot" and snap["items"] == []

        async def writer(w):
            c = await ControlPlaneClient(native).connect()
            for i in range(50):
                await c.put(f"wo/{w}/{i}", str(i).encode())
            await c.close()

        await asyncio.gather(*(writer(w) for w in range(8)))
        evs = [await st.__anext__() for _ in range(400)]
        revs = [e["rev"] for e in evs]
        assert revs == sorted(revs) and len(set(revs)) == 400
        for w in range(8):  # per-writer order preserved
            mine = [int(e["key"].rsplit("/", 1)[1]) for e in evs if e["key"].startswith(f"wo/{w}/")]
            assert mine == list(range(50))
        await st.cancel()
        await watcher.close()

    run(main())


def test_cancelled_pop_waiter_does_not_swallow_messages(native):
    async def main():
        c = await ControlPlaneClient(native).connect()
        st = await c.stream("q_pop", queue="cq", timeout=30.0)  # a long pop ...
        await asyncio.sleep(0.05)
        await st.cancel()  # ... abandoned by its caller
        await c.q_push("cq", b"m")
        m = await c.q_pop("cq", timeout=2)
        assert m is not None and m["data"] == b"m"
        await c.close()

    run(main())


def test_malformed_frame_drops_only_that_connection(native):
    host, port = native.rsplit(":", 1)
    s = socket.create_connection((host, int(port)))
    s.sendall(struct.pack(">I", 3) + b"\xc1\xc1\xc1")  # 0xc1 is never valid msgpack
    s.settimeout(5)
    assert s.recv(16) == b""  # server closed it
    s.close()

    async def main():
        c = await ControlPlaneClient(native).connect()
        await c.put("alive", b"1")
        assert await c.get("alive") == b"1"
        st = await c.call("stats")
        assert st["server"] == "native"
        await c.close()

    run(main())


def test_server_exits_with_its_parent(native):
    """A child dx-ctrld started with --exit-with-parent (the bench's rank 0
    control plane) ends when its parent is killed outright."""
    import os
    import signal
    import subprocess
    import sys
    import time

    code = ("import sys; from dynamo_exp_amd.runtime.control_plane import NativeServerProcess as N; "
            "s = N('127.0.0.1', 0, exit_with_parent=True).start(); print(s.proc.pid, flush=True); sys.stdin.readline()")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    parent = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stdin=subprocess.PIPE,
                              text=True, cwd=root)
    child = int(parent.stdout.readline())
    os.kill(parent.pid, signal.SIGKILL)
    parent.wait(10)
    deadline = time.monotonic() + 10
    while time.monotonic() < deadline:
        try:
            os.kill(child, 0)
        except ProcessLookupError:
            return
        try:  # reap it if it became our zombie
            os.waitpid(child, os.WNOHANG)
        except ChildProcessError:
            pass
        time.sleep(0.05)
    os.kill(child, signal.SIGKILL)
    raise AssertionError("dx-ctrld outlived its parent")
