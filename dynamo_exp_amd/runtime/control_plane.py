"""In-tree control plane: the etcd + NATS replacement.

One asyncio TCP server (`ctrld`) provides everything the reference takes from
etcd and NATS/JetStream:

* revisioned key-value store with **leases** (TTL + keep-alive; revoke or
  expiry deletes every key bound to the lease), transactional
  create-if-absent (`kv_create`, reference transports/etcd.rs:170-198) and
  **prefix watches** that start with a consistent snapshot
  (`kv_get_and_watch_prefix`, etcd.rs:309);
* **pub/sub** with NATS subject wildcards (`*` one token, `>` the rest) for
  KV events, load metrics, hit-rate events;
* a durable **work queue** with explicit ack, redelivery after `ack_wait` and
  `num_pending` (JetStream pull consumer used as the prefill queue,
  examples/llm/utils/nats_queue.py);
* a small **blob store** (NATS object store for model-card files).

Wire: u32-BE-length-prefixed msgpack frames, one multiplexed connection per
client; request ids tag responses and stream items.  The server is
single-threaded asyncio, so every operation is atomic w.r.t. the others.
Run standalone: ``python -m dynamo_exp_amd.runtime.control_plane --port 4850``.
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import itertools
import logging
import os
import subprocess
import threading
import time
from dataclasses import dataclass, field
from typing import Any, AsyncIterator

from .wire import pack, read_frame

log = logging.getLogger("dynamo_exp_amd.ctrld")

DEFAULT_ADDR = "127.0.0.1:4850"


def default_address() -> str:
    return os.environ.get("DX_CONTROL_PLANE", DEFAULT_ADDR)


def subject_matches(pattern: str, subject: str) -> bool:
    if pattern == subject:
        return True
    p, s = pattern.split("."), subject.split(".")
    for i, tok in enumerate(p):
        if tok == ">":
            return len(s) > i
        if i >= len(s):
            return False
        if tok != "*" and tok != s[i]:
            return False
    return len(p) == len(s)


@dataclass
class _Lease:
    id: int
    ttl: float
    deadline: float
    keys: set = field(default_factory=set)


@dataclass
class _QMsg:
    seq: int
    data: bytes
    deliveries: int = 0
    deadline: float = 0.0


class _Queue:
    def __init__(self):
        self.ready: collections.deque[_QMsg] = collections.deque()
        self.inflight: dict[int, _QMsg] = {}
        self.waiters: collections.deque[asyncio.Future] = collections.deque()
        self.seq = itertools.count(1)


class ControlPlaneServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 4850):
        self.host, self.port = host, port
        self.kv: dict[str, tuple[bytes, int, int | None]] = {}  # key -> (value, mod_rev, lease)
        self.rev = 0
        self.leases: dict[int, _Lease] = {}
        self._lease_ids = itertools.count(0x1000 + (os.getpid() & 0xFFF) * 0x10000)
        self.watchers: dict[int, tuple[str, asyncio.Queue]] = {}
        self.subs: dict[int, tuple[str, asyncio.Queue]] = {}
        self._wid = itertools.count(1)
        self.queues: dict[str, _Queue] = collections.defaultdict(_Queue)
        self.blobs: dict[str, dict[str, tuple[bytes, float | None]]] = collections.defaultdict(dict)
        self._server: asyncio.AbstractServer | None = None
        self._tasks: list[asyncio.Task] = []
        self.stats = collections.Counter()

    # ----------------------------------------------------------------- lifecycle
    async def start(self) -> "ControlPlaneServer":
        self._server = await asyncio.start_server(self._handle, self.host, self.port, limit=1 << 24)
        self.port = self._server.sockets[0].getsockname()[1]
        self._tasks.append(asyncio.create_task(self._reaper()))
        log.info("control plane listening on %s:%d", self.host, self.port)
        return self

    @property
    def address(self) -> str:
        return f"{self.host}:{self.port}"

    async def stop(self) -> None:
        for t in self._tasks:
            t.cancel()
        if self._server is not None:
            self._server.close()
            await self._server.wait_closed()

    async def _reaper(self) -> None:
        while True:
            await asyncio.sleep(0.05)
            now = time.monotonic()
            for lid in [l.id for l in self.leases.values() if l.deadline < now]:
                log.info("lease %x expired", lid)
                self._revoke(lid)
            for name, q in self.queues.items():
                for seq in [s for s, m in q.inflight.items() if m.deadline < now]:
                    m = q.inflight.pop(seq)
                    q.ready.appendleft(m)
                    self._q_wake(q)
            for bucket in self.blobs.values():
                for k in [k for k, (_, exp) in bucket.items() if exp is not None and exp < now]:
                    del bucket[k]

    # ----------------------------------------------------------------- kv
    def _notify(self, kind: str, key: str, value: bytes | None, rev: int) -> None:
        ev = {"type": kind, "key": key, "value": value, "rev": rev}
        for prefix, q in self.watchers.values():
            if key.startswith(prefix):
                q.put_nowait(ev)

    def _put(self, key: str, value: bytes, lease: int | None) -> int:
        if lease is not None:
            if lease not in self.leases:
                raise KeyError(f"lease {lease:x} not found")
            self.leases[lease].keys.add(key)
        old = self.kv.get(key)
        if old is not None and old[2] is not None and old[2] != lease and old[2] in self.leases:
            self.leases[old[2]].keys.discard(key)
        self.rev += 1
        self.kv[key] = (value, self.rev, lease)
        self._notify("put", key, value, self.rev)
        return self.rev

    def _delete(self, key: str) -> int:
        old = self.kv.pop(key, None)
        if old is None:
            return 0
        if old[2] is not None and old[2] in self.leases:
            self.leases[old[2]].keys.discard(key)
        self.rev += 1
        self._notify("delete", key, None, self.rev)
        return 1

    def _revoke(self, lid: int) -> int:
        lease = self.leases.pop(lid, None)
        if lease is None:
            return 0
        n = 0
        for k in list(lease.keys):
            cur = self.kv.get(k)
            if cur is not None and cur[2] == lid:
                n += self._delete(k)
        return n

    # ----------------------------------------------------------------- queue
    def _q_wake(self, q: _Queue) -> None:
        while q.waiters and q.ready:
            fut = q.waiters.popleft()
            if not fut.done():
                fut.set_result(True)
                return

    # ----------------------------------------------------------------- dispatch
    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        streams: dict[int, asyncio.Task] = {}
        wlock = asyncio.Lock()

        async def send(obj):
            async with wlock:
                writer.write(pack(obj))
                await writer.drain()

        try:
            while True:
                msg = await read_frame(reader)
                rid, op = msg.get("id"), msg.get("op")
                self.stats[op] += 1
                if op == "cancel":
                    t = streams.pop(msg.get("target"), None)
                    if t:
                        t.cancel()
                    continue
                if op in ("watch", "subscribe", "q_pop"):
                    streams[rid] = asyncio.create_task(self._stream_op(op, rid, msg, send, streams))
                    continue
                try:
                    res = self._op(op, msg)
                    await send({"id": rid, "ok": True, "result": res})
                except Exception as e:  # noqa: BLE001
                    await send({"id": rid, "ok": False, "error": f"{type(e).__name__}: {e}"})
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            for t in streams.values():
                t.cancel()
            try:
                writer.close()
            except RuntimeError:  # loop already closed (server torn down with clients attached)
                pass

    def _op(self, op: str, m: dict) -> Any:
        if op == "ping":
            return {"rev": self.rev, "time": time.time()}
        if op == "put":
            return {"rev": self._put(m["key"], m["value"], m.get("lease"))}
        if op == "create":
            if m["key"] in self.kv:
                return {"ok": False, "rev": self.kv[m["key"]][1]}
            return {"ok": True, "rev": self._put(m["key"], m["value"], m.get("lease"))}
        if op == "create_or_validate":
            cur = self.kv.get(m["key"])
            if cur is None:
                return {"ok": True, "rev": self._put(m["key"], m["value"], m.get("lease"))}
            return {"ok": cur[0] == m["value"], "rev": cur[1]}
        if op == "get":
            cur = self.kv.get(m["key"])
            return None if cur is None else {"value": cur[0], "rev": cur[1], "lease": cur[2]}
        if op == "get_prefix":
            p = m["prefix"]
            return {"items": [[k, v[0], v[1]] for k, v in sorted(self.kv.items()) if k.startswith(p)], "rev": self.rev}
        if op == "delete":
            return {"deleted": self._delete(m["key"])}
        if op == "delete_prefix":
            p = m["prefix"]
            return {"deleted": sum(self._delete(k) for k in [k for k in self.kv if k.startswith(p)])}
        if op == "lease_grant":
            lid = next(self._lease_ids)
            ttl = float(m.get("ttl", 10.0))
            self.leases[lid] = _Lease(lid, ttl, time.monotonic() + ttl)
            return {"lease": lid, "ttl": ttl}
        if op == "lease_keepalive":
            l = self.leases.get(m["lease"])
            if l is None:
                return {"ok": False}
            l.deadline = time.monotonic() + l.ttl
            return {"ok": True, "ttl": l.ttl}
        if op == "lease_revoke":
            return {"deleted": self._revoke(m["lease"])}
        if op == "lease_alive":
            return {"ok": m["lease"] in self.leases}
        if op == "publish":
            subj = m["subject"]
            n = 0
            for pat, q in self.subs.values():
                if subject_matches(pat, subj):
                    q.put_nowait({"subject": subj, "data": m["data"]})
                    n += 1
            return {"delivered": n}
        if op == "q_push":
            q = self.queues[m["queue"]]
            msg = _QMsg(next(q.seq), m["data"])
            q.ready.append(msg)
            self._q_wake(q)
            return {"seq": msg.seq}
        if op == "q_ack":
            q = self.queues[m["queue"]]
            return {"ok": q.inflight.pop(m["seq"], None) is not None}
        if op == "q_nak":
            q = self.queues[m["queue"]]
            msg = q.inflight.pop(m["seq"], None)
            if msg is not None:
                q.ready.appendleft(msg)
                self._q_wake(q)
            return {"ok": msg is not None}
        if op == "q_size":
            q = self.queues[m["queue"]]
            return {"pending": len(q.ready), "inflight": len(q.inflight)}
        if op == "blob_put":
            ttl = m.get("ttl")
            self.blobs[m["bucket"]][m["key"]] = (m["data"], time.monotonic() + ttl if ttl else None)
            return {"ok": True}
        if op == "blob_get":
            b = self.blobs.get(m["bucket"], {}).get(m["key"])
            return None if b is None else b[0]
        if op == "blob_list":
            return sorted(self.blobs.get(m["bucket"], {}).keys())
        if op == "blob_delete":
            return {"ok": self.blobs.get(m["bucket"], {}).pop(m["key"], None) is not None}
        if op == "stats":
            return {"keys": len(self.kv), "leases": len(self.leases), "rev": self.rev, "watchers": len(self.watchers),
                    "subs": len(self.subs), "queues": {k: len(v.ready) for k, v in self.queues.items()},
                    "ops": dict(self.stats)}
        raise ValueError(f"unknown op {op}")

    async def _stream_op(self, op: str, rid: int, m: dict, send, streams) -> None:
        try:
            if op == "watch":
                q: asyncio.Queue = asyncio.Queue()
                wid = next(self._wid)
                p = m["prefix"]
                snap = [[k, v[0], v[1]] for k, v in sorted(self.kv.items()) if k.startswith(p)]
                self.watchers[wid] = (p, q)
                try:
                    await send({"id": rid, "ok": True, "item": {"type": "snapshot", "items": snap, "rev": self.rev}})
                    while True:
                        ev = await q.get()
                        await send({"id": rid, "ok": True, "item": ev})
                finally:
                    self.watchers.pop(wid, None)
            elif op == "subscribe":
                q = asyncio.Queue()
                sid = next(self._wid)
                self.subs[sid] = (m["subject"], q)
                try:
                    await send({"id": rid, "ok": True, "item": {"type": "subscribed"}})
                    while True:
                        item = await q.get()
                        await send({"id": rid, "ok": True, "item": item})
                finally:
                    self.subs.pop(sid, None)
            elif op == "q_pop":
                q = self.queues[m["queue"]]
                timeout = float(m.get("timeout", 1.0))
                ack_wait = float(m.get("ack_wait", 30.0))
                end = time.monotonic() + timeout
                while not q.ready:
                    rem = end - time.monotonic()
                    if rem <= 0:
                        break
                    fut = asyncio.get_running_loop().create_future()
                    q.waiters.append(fut)
                    try:
                        await asyncio.wait_for(fut, rem)
                    except asyncio.TimeoutError:
                        pass
                if q.ready:
                    msg = q.ready.popleft()
                    msg.deliveries += 1
                    msg.deadline = time.monotonic() + ack_wait
                    q.inflight[msg.seq] = msg
                    await send({"id": rid, "ok": True, "result": {"seq": msg.seq, "data": msg.data,
                                                                  "deliveries": msg.deliveries}})
                else:
                    await send({"id": rid, "ok": True, "result": None})
                self._q_wake(q)
        except asyncio.CancelledError:
            pass
        except (ConnectionError, RuntimeError):
            pass
        finally:
            streams.pop(rid, None)


# ===================================================================== client
class ControlPlaneError(Exception):
    pass


class Stream:
    def __init__(self, client: "ControlPlaneClient", rid: int):
        self.client, self.rid = client, rid
        self.queue: asyncio.Queue = asyncio.Queue()
        self.closed = False

    def __aiter__(self):
        return self

    async def __anext__(self):
        if self.closed and self.queue.empty():
            raise StopAsyncIteration
        item = await self.queue.get()
        if item is None:
            self.closed = True
            raise StopAsyncIteration
        return item

    async def cancel(self) -> None:
        if not self.closed:
            self.closed = True
            self.client._streams.pop(self.rid, None)
            try:
                await self.client._send({"id": 0, "op": "cancel", "target": self.rid})
            except Exception:
                pass
            self.queue.put_nowait(None)


class ControlPlaneClient:
    """Asyncio client; one multiplexed connection."""

    def __init__(self, address: str | None = None):
        self.address = address or default_address()
        self._ids = itertools.count(1)
        self._pending: dict[int, asyncio.Future] = {}
        self._streams: dict[int, Stream] = {}
        self._reader = self._writer = None
        self._rtask = None
        self._wlock = asyncio.Lock()
        self.connected = False
        self.on_disconnect = []

    async def connect(self, timeout: float = 10.0) -> "ControlPlaneClient":
        host, port = self.address.rsplit(":", 1)
        end = time.monotonic() + timeout
        while True:
            try:
                self._reader, self._writer = await asyncio.open_connection(host, int(port), limit=1 << 24)
                break
            except OSError:
                if time.monotonic() > end:
                    raise ControlPlaneError(f"cannot reach control plane at {self.address}")
                await asyncio.sleep(0.1)
        self.connected = True
        self._rtask = asyncio.create_task(self._read_loop())
        return self

    async def close(self) -> None:
        if self._writer is not None:
            self._writer.close()
        if self._rtask is not None:
            self._rtask.cancel()
        self.connected = False

    async def _read_loop(self) -> None:
        try:
            while True:
                msg = await read_frame(self._reader)
                rid = msg.get("id")
                if "item" in msg:
                    st = self._streams.get(rid)
                    if st is not None:
                        st.queue.put_nowait(msg["item"])
                    continue
                fut = self._pending.pop(rid, None)
                if fut is not None and not fut.done():
                    if msg.get("ok"):
                        fut.set_result(msg.get("result"))
                    else:
                        fut.set_exception(ControlPlaneError(msg.get("error")))
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.CancelledError):
            pass
        finally:
            self.connected = False
            for fut in self._pending.values():
                if not fut.done():
                    fut.set_exception(ControlPlaneError("control plane connection lost"))
            for st in self._streams.values():
                st.queue.put_nowait(None)
            for cb in self.on_disconnect:
                try:
                    cb()
                except Exception:
                    pass

    async def _send(self, obj) -> None:
        async with self._wlock:
            self._writer.write(pack(obj))
            await self._writer.drain()

    async def call(self, op: str, **kw) -> Any:
        if not self.connected:
            raise ControlPlaneError("not connected")
        rid = next(self._ids)
        fut = asyncio.get_running_loop().create_future()
        self._pending[rid] = fut
        await self._send({"id": rid, "op": op, **kw})
        return await fut

    async def stream(self, op: str, **kw) -> Stream:
        rid = next(self._ids)
        st = Stream(self, rid)
        self._streams[rid] = st
        await self._send({"id": rid, "op": op, **kw})
        return st

    # ---- kv
    async def put(self, key: str, value: bytes, lease: int | None = None) -> int:
        return (await self.call("put", key=key, value=value, lease=lease))["rev"]

    async def create(self, key: str, value: bytes, lease: int | None = None) -> bool:
        return (await self.call("create", key=key, value=value, lease=lease))["ok"]

    async def create_or_validate(self, key: str, value: bytes, lease: int | None = None) -> bool:
        return (await self.call("create_or_validate", key=key, value=value, lease=lease))["ok"]

    async def get(self, key: str) -> bytes | None:
        r = await self.call("get", key=key)
        return None if r is None else r["value"]

    async def get_prefix(self, prefix: str) -> list[tuple[str, bytes]]:
        r = await self.call("get_prefix", prefix=prefix)
        return [(k, v) for k, v, _ in r["items"]]

    async def delete(self, key: str) -> int:
        return (await self.call("delete", key=key))["deleted"]

    async def delete_prefix(self, prefix: str) -> int:
        return (await self.call("delete_prefix", prefix=prefix))["deleted"]

    async def watch_prefix(self, prefix: str) -> Stream:
        """First item: {'type':'snapshot','items':[[k,v,rev]...]}; then put/delete events."""
        return await self.stream("watch", prefix=prefix)

    # ---- leases
    async def lease_grant(self, ttl: float) -> int:
        return (await self.call("lease_grant", ttl=ttl))["lease"]

    async def lease_keepalive(self, lease: int) -> bool:
        return (await self.call("lease_keepalive", lease=lease))["ok"]

    async def lease_revoke(self, lease: int) -> int:
        return (await self.call("lease_revoke", lease=lease))["deleted"]

    async def lease_alive(self, lease: int) -> bool:
        return (await self.call("lease_alive", lease=lease))["ok"]

    # ---- pub/sub
    async def publish(self, subject: str, data: bytes) -> int:
        return (await self.call("publish", subject=subject, data=data))["delivered"]

    async def subscribe(self, subject: str) -> Stream:
        st = await self.stream("subscribe", subject=subject)
        first = await st.queue.get()  # 'subscribed' ack: subscription is live
        assert first is None or first.get("type") == "subscribed"
        return st

    # ---- queue
    async def q_push(self, queue: str, data: bytes) -> int:
        return (await self.call("q_push", queue=queue, data=data))["seq"]

    async def q_pop(self, queue: str, timeout: float = 1.0, ack_wait: float = 30.0):
        rid = next(self._ids)
        fut = asyncio.get_running_loop().create_future()
        self._pending[rid] = fut
        await self._send({"id": rid, "op": "q_pop", "queue": queue, "timeout": timeout, "ack_wait": ack_wait})
        return await fut

    async def q_ack(self, queue: str, seq: int) -> bool:
        return (await self.call("q_ack", queue=queue, seq=seq))["ok"]

    async def q_nak(self, queue: str, seq: int) -> bool:
        return (await self.call("q_nak", queue=queue, seq=seq))["ok"]

    async def q_size(self, queue: str) -> int:
        return (await self.call("q_size", queue=queue))["pending"]

    # ---- blobs
    async def blob_put(self, bucket: str, key: str, data: bytes, ttl: float | None = None) -> None:
        await self.call("blob_put", bucket=bucket, key=key, data=data, ttl=ttl)

    async def blob_get(self, bucket: str, key: str) -> bytes | None:
        return await self.call("blob_get", bucket=bucket, key=key)

    async def blob_list(self, bucket: str) -> list[str]:
        return await self.call("blob_list", bucket=bucket)


# ===================================================================== helpers
class BackgroundServer:
    """Run a ControlPlaneServer on its own thread (tests, single-node bring-up)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.loop = asyncio.new_event_loop()
        self.server = ControlPlaneServer(host, port)
        self._ready = threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True, name="dx-ctrld")

    def _run(self):
        asyncio.set_event_loop(self.loop)
        self.loop.run_until_complete(self.server.start())
        self._ready.set()
        self.loop.run_forever()

    def start(self) -> "BackgroundServer":
        self.thread.start()
        self._ready.wait(10)
        return self

    @property
    def address(self) -> str:
        return self.server.address

    def stop(self):
        fut = asyncio.run_coroutine_threadsafe(self.server.stop(), self.loop)
        try:
            fut.result(5)
        except Exception:
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)


class SyncControlPlaneClient:
    """Blocking facade over ControlPlaneClient (own event loop thread) for
    non-async code such as the engine thread and the bench."""

    def __init__(self, address: str | None = None):
        self.loop = asyncio.new_event_loop()
        self._t = threading.Thread(target=self.loop.run_forever, daemon=True, name="dx-cp-client")
        self._t.start()
        self.client = ControlPlaneClient(address)
        self.run(self.client.connect())

    def run(self, coro, timeout: float | None = 60.0):
        return asyncio.run_coroutine_threadsafe(coro, self.loop).result(timeout)

    def __getattr__(self, name):
        fn = getattr(self.client, name)
        if not asyncio.iscoroutinefunction(fn):
            return fn

        def wrapper(*a, **kw):
            return self.run(fn(*a, **kw))

        return wrapper

    def subscribe_callback(self, subject: str, cb) -> None:
        """Invoke cb(subject, data) on the client thread for each message."""

        async def pump():
            st = await self.client.subscribe(subject)
            async for item in st:
                try:
                    cb(item["subject"], item["data"])
                except Exception:
                    log.exception("subscriber callback failed")

        self.run(asyncio.sleep(0))
        fut = asyncio.run_coroutine_threadsafe(pump(), self.loop)
        return fut

    def close(self):
        try:
            self.run(self.client.close(), timeout=5)
        except Exception:
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)


def native_server_binary() -> str | None:
    """Path of the native server (csrc/ctrld -> bin/dx-ctrld) if it is built."""
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin", "dx-ctrld")
    return p if os.access(p, os.X_OK) else None


def use_native_server() -> bool:
    """`DX_CTRLD=native|python` (default: native when built)."""
    want = os.environ.get("DX_CTRLD", "auto").lower()
    if want == "python":
        return False
    if want == "native" and native_server_binary() is None:
        raise RuntimeError("DX_CTRLD=native but bin/dx-ctrld is not built (python -m dynamo_exp_amd.build_native)")
    return native_server_binary() is not None


class NativeServerProcess:
    """The native control-plane server (`dx-ctrld`, same protocol as
    ControlPlaneServer) as a child process."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, exit_with_parent: bool = False):
        self.host, self.port = host, port
        # SIGTERM to the server when the thread that started it ends (Linux
        # parent-death signal): start it from the main thread
        self.exit_with_parent = exit_with_parent
        self.proc: subprocess.Popen | None = None

    def start(self, timeout: float = 10.0) -> "NativeServerProcess":
        exe = native_server_binary()
        if exe is None:
            raise RuntimeError("bin/dx-ctrld is not built")
        cmd = [exe, "--host", self.host, "--port", str(self.port)]
        if self.exit_with_parent:
            cmd += ["--parent-pid", str(os.getpid())]
        self.proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stdin=subprocess.DEVNULL, text=True)
        line = ""
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            line = self.proc.stdout.readline()
            if line.startswith("ctrld listening on") or self.proc.poll() is not None:
                break
        if not line.startswith("ctrld listening on"):
            self.stop()
            raise RuntimeError(f"dx-ctrld failed to start: {line!r}")
        self.port = int(line.strip().rsplit(":", 1)[1])
        return self

    @property
    def address(self) -> str:
        host = "127.0.0.1" if self.host in ("0.0.0.0", "") else self.host
        return f"{host}:{self.port}"

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(5)


def main(argv=None):
    ap = argparse.ArgumentParser(description="dynamo_exp_amd control plane (etcd+NATS replacement)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=int(default_address().rsplit(":", 1)[1]))
    ap.add_argument("--python", action="store_true", help="run the asyncio server instead of the native dx-ctrld")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    if not a.python and use_native_server():
        # run the native server as a child (no exec: keep one supervisor semantics)
        proc = subprocess.Popen([native_server_binary(), "--host", a.host, "--port", str(a.port)])
        try:
            raise SystemExit(proc.wait())
        except KeyboardInterrupt:
            proc.terminate()
            raise SystemExit(proc.wait())

    async def run():
        s = await ControlPlaneServer(a.host, a.port).start()
        print(f"ctrld listening on {a.host}:{s.port}", flush=True)
        await asyncio.Event().wait()

    asyncio.run(run())


if __name__ == "__main__":
    main()
