"""Bucketed key-value store abstraction (reference lib/llm/src/key_value_store.rs:37-200,
key_value_store/{mem,etcd,nats}.rs).

A `KeyValueStore` hands out buckets (optionally with an item TTL); a bucket
supports versioned `insert`, `get`, `delete`, `entries` and `watch` (existing
entries first, then live puts).  Two backends:

* `MemoryStorage`   -- in-process (tests, static single-process mode);
* `ControlPlaneStorage` -- keys `kvstore/{bucket}/{key}` on the in-tree
  control plane; a TTL bucket attaches each item to a fresh lease of that TTL,
  so items disappear unless re-published (NATS KV `max_age` semantics).

`KeyValueStoreManager` adds JSON (de)serialisation of versioned objects,
`publish` (create-or-update by revision) and `publish_until_cancelled`.
Insert semantics: absent key -> Created(rev); same revision -> Exists(rev);
otherwise overwritten -> Created(rev).
"""
from __future__ import annotations

import abc
import asyncio
import json
import time
from dataclasses import dataclass
from typing import Any, AsyncIterator

PREFIX = "kvstore/"


@dataclass(frozen=True)
class StorageOutcome:
    kind: str  # "created" | "exists"
    revision: int


class KeyValueBucket(abc.ABC):
    @abc.abstractmethod
    async def insert(self, key: str, value: str, revision: int) -> StorageOutcome: ...

    @abc.abstractmethod
    async def get(self, key: str) -> bytes | None: ...

    @abc.abstractmethod
    async def delete(self, key: str) -> None: ...

    @abc.abstractmethod
    async def entries(self) -> dict[str, bytes]: ...

    @abc.abstractmethod
    def watch(self) -> AsyncIterator[bytes]: ...


class KeyValueStore(abc.ABC):
    @abc.abstractmethod
    async def get_or_create_bucket(self, name: str, ttl: float | None = None) -> KeyValueBucket: ...

    @abc.abstractmethod
    async def get_bucket(self, name: str) -> KeyValueBucket | None: ...


# ------------------------------------------------------------------ memory
class _MemBucket(KeyValueBucket):
    def __init__(self, name: str, ttl: float | None):
        self.name, self.ttl = name, ttl
        self.data: dict[str, tuple[int, str, float]] = {}
        self.watchers: list[asyncio.Queue] = []

    def _expire(self):
        if self.ttl:
            now = time.monotonic()
            for k in [k for k, (_, _, t) in self.data.items() if now - t > self.ttl]:
                del self.data[k]

    async def insert(self, key, value, revision):
        self._expire()
        cur = self.data.get(key)
        if cur is not None and cur[0] == revision:
            return StorageOutcome("exists", revision)
        self.data[key] = (revision, value, time.monotonic())
        for q in self.watchers:
            q.put_nowait(value.encode())
        return StorageOutcome("created", revision)

    async def get(self, key):
        self._expire()
        v = self.data.get(key)
        return v[1].encode() if v else None

    async def delete(self, key):
        self.data.pop(key, None)

    async def entries(self):
        self._expire()
        return {k: v.encode() for k, (_, v, _) in self.data.items()}

    async def watch(self):
        q: asyncio.Queue = asyncio.Queue()
        self.watchers.append(q)
        try:
            while True:
                yield await q.get()
        finally:
            self.watchers.remove(q)


class MemoryStorage(KeyValueStore):
    def __init__(self):
        self.buckets: dict[str, _MemBucket] = {}

    async def get_or_create_bucket(self, name, ttl=None):
        b = self.buckets.get(name)
        if b is None:
            b = self.buckets[name] = _MemBucket(name, ttl)
        return b

    async def get_bucket(self, name):
        return self.buckets.get(name)


# ------------------------------------------------------------------ control plane
class _CPBucket(KeyValueBucket):
    def __init__(self, cp, name: str, ttl: float | None):
        self.cp, self.name, self.ttl = cp, name, ttl
        self.prefix = f"{PREFIX}{name}/"

    async def insert(self, key, value, revision):
        raw = await self.cp.get(self.prefix + key)
        if raw is not None and json.loads(raw)["rev"] == revision:
            return StorageOutcome("exists", revision)
        lease = await self.cp.lease_grant(self.ttl) if self.ttl else None
        await self.cp.put(self.prefix + key, json.dumps({"rev": revision, "value": value}).encode(), lease=lease)
        return StorageOutcome("created", revision)

    async def get(self, key):
        raw = await self.cp.get(self.prefix + key)
        return json.loads(raw)["value"].encode() if raw is not None else None

    async def delete(self, key):
        await self.cp.delete(self.prefix + key)

    async def entries(self):
        return {k[len(self.prefix):]: json.loads(v)["value"].encode() for k, v in await self.cp.get_prefix(self.prefix)}

    async def watch(self):
        st = await self.cp.watch_prefix(self.prefix)
        await st.__anext__()  # initial snapshot (callers read entries() first)
        async for ev in st:
            if ev["type"] == "put":
                yield json.loads(ev["value"])["value"].encode()


class ControlPlaneStorage(KeyValueStore):
    def __init__(self, cp):
        self.cp = cp
        self._buckets: dict[str, _CPBucket] = {}

    async def get_or_create_bucket(self, name, ttl=None):
        b = self._buckets.get(name)
        if b is None:
            b = self._buckets[name] = _CPBucket(self.cp, name, ttl)
        return b

    async def get_bucket(self, name):
        if name in self._buckets:
            return self._buckets[name]
        if await self.cp.get_prefix(f"{PREFIX}{name}/"):
            return await self.get_or_create_bucket(name)
        return None


# ------------------------------------------------------------------ manager
class KeyValueStoreManager:
    """JSON objects with a `revision` attribute (or dict key)."""

    def __init__(self, store: KeyValueStore):
        self.store = store

    async def load(self, bucket: str, key: str) -> Any | None:
        b = await self.store.get_bucket(bucket)
        if b is None:
            return None
        raw = await b.get(key)
        return json.loads(raw) if raw is not None else None

    async def publish(self, bucket: str, key: str, obj: dict, ttl: float | None = None) -> StorageOutcome:
        b = await self.store.get_or_create_bucket(bucket, ttl)
        out = await b.insert(key, json.dumps(obj, sort_keys=True), int(obj.get("revision", 0)))
        obj["revision"] = out.revision
        return out

    async def watch(self, bucket: str, ttl: float | None = None) -> AsyncIterator[Any]:
        b = await self.store.get_or_create_bucket(bucket, ttl)
        it = b.watch()
        for v in (await b.entries()).values():
            yield json.loads(v)
        async for v in it:
            yield json.loads(v)

    def publish_until_cancelled(self, bucket: str, key: str, obj: dict, interval: float,
                                ttl: float | None = None) -> asyncio.Task:
        async def loop():
            try:
                while True:
                    obj["revision"] = int(obj.get("revision", 0)) + 1
                    await self.publish(bucket, key, obj, ttl)
                    await asyncio.sleep(interval)
            finally:
                b = await self.store.get_bucket(bucket)
                if b is not None:
                    await b.delete(key)

        return asyncio.create_task(loop())
