"""DistributedRuntime: namespaces, components, endpoints, leases, discovery.

API parity with the reference Python bindings (`dynamo._core`,
lib/bindings/python/src/dynamo/_core.pyi):

    drt = await DistributedRuntime.create()              # or DistributedRuntime(loop)
    ep = drt.namespace("dynamo").component("Worker").endpoint("generate")
    await ep.component.create_service()
    await ep.serve_endpoint(handler)                     # async-generator handler
    client = await ep.client(); await client.wait_for_instances()
    async for out in await client.round_robin(req): ...  # or random / direct(req, id)

Naming (reference lib/runtime/src/component.rs:153-286):
  registration key  {ns}/components/{comp}/{ep}:{lease_hex}   (value: instance info)
  event subjects    namespace.{ns}[.component.{comp}].{event}
The instance id of an endpoint is its lease id.  The primary lease (TTL 10 s,
keep-alive every ttl/2) dies with the process: when the keep-alive fails the
runtime token fires and the process shuts down (etcd/lease.rs:30-121).
"""
from __future__ import annotations

import asyncio
import json
import logging
import random
import re
from dataclasses import dataclass
from typing import Any, AsyncIterator, Callable

from .context import Context
from .control_plane import ControlPlaneClient, default_address
from .transport import ConnectionPool, EndpointError, EndpointServer, ResponseStream, call_endpoint, scrape_stats

log = logging.getLogger("dynamo_exp_amd.runtime")


def slugify(s: str) -> str:
    """Subject-safe name (reference lib/runtime/src/slug.rs)."""
    s = s.lower()
    s = re.sub(r"[^a-z0-9_\-]", "_", s)
    return s


class Lease:
    def __init__(self, drt: "DistributedRuntime", lease_id: int, ttl: float):
        self.drt, self.id, self.ttl = drt, lease_id, ttl
        self._task: asyncio.Task | None = None
        self.valid = True
        self.on_lost: list[Callable[[], None]] = []

    def start(self) -> "Lease":
        self._task = asyncio.create_task(self._keepalive())
        return self

    async def _keepalive(self):
        try:
            while self.valid:
                await asyncio.sleep(self.ttl / 2 if self.ttl > 1 else self.ttl / 3)
                ok = await self.drt.cp.lease_keepalive(self.id)
                if not ok:
                    break
        except asyncio.CancelledError:
            return
        except Exception:
            log.warning("lease %x keep-alive failed", self.id)
        self.valid = False
        for cb in self.on_lost:
            try:
                cb()
            except Exception:
                pass

    def is_valid(self) -> bool:
        return self.valid

    async def revoke(self) -> None:
        self.valid = False
        if self._task:
            self._task.cancel()
        try:
            await self.drt.cp.lease_revoke(self.id)
        except Exception:
            pass
        for cb in self.on_lost:
            try:
                cb()
            except Exception:
                pass

    def __repr__(self):
        return f"Lease({self.id:x}, ttl={self.ttl})"


class DistributedRuntime:
    PRIMARY_LEASE_TTL = 10.0

    def __init__(self, loop: asyncio.AbstractEventLoop | None = None, address: str | None = None,
                 is_static: bool = False):
        self.loop = loop
        self.address = address or default_address()
        self.is_static = is_static
        self.cp: ControlPlaneClient | None = None
        self.primary_lease: Lease | None = None
        self.server = EndpointServer()
        self.pool = ConnectionPool()
        self.shutdown_event = asyncio.Event()
        self._served: list[str] = []
        self._leases: list[Lease] = []

    @classmethod
    async def create(cls, address: str | None = None, is_static: bool = False) -> "DistributedRuntime":
        drt = cls(asyncio.get_running_loop(), address, is_static)
        await drt.init()
        return drt

    async def init(self) -> "DistributedRuntime":
        self.cp = await ControlPlaneClient(self.address).connect()
        if not self.is_static:
            self.primary_lease = await self.create_lease(self.PRIMARY_LEASE_TTL)
            self.primary_lease.on_lost.append(self._lease_lost)
        self.cp.on_disconnect.append(self._lease_lost)
        return self

    def _lease_lost(self):
        if not self.shutdown_event.is_set():
            log.error("primary lease / control plane lost: shutting down")
            self.shutdown_event.set()

    async def create_lease(self, ttl: float) -> Lease:
        lid = await self.cp.lease_grant(ttl)
        lease = Lease(self, lid, ttl).start()
        self._leases.append(lease)
        return lease

    def namespace(self, name: str) -> "Namespace":
        return Namespace(self, name)

    def shutdown(self) -> None:
        self.shutdown_event.set()

    async def close(self, drain_timeout: float = 30.0) -> None:
        for path in list(self._served):
            await self.server.drain(path, drain_timeout)
        for lease in self._leases:
            if lease.valid:
                await lease.revoke()
        await self.server.stop()
        await self.pool.close()
        if self.cp is not None:
            await self.cp.close()

    # ---- convenience for KV helpers
    def etcd_client(self) -> ControlPlaneClient:
        return self.cp


class Namespace:
    def __init__(self, drt: DistributedRuntime, name: str):
        self.drt, self.name = drt, name

    def component(self, name: str) -> "Component":
        return Component(self, name)

    def subject(self, event: str) -> str:
        return f"namespace.{self.name}.{event}"

    async def publish(self, event: str, payload: Any) -> None:
        await self.drt.cp.publish(self.subject(event), _enc(payload))

    async def subscribe(self, event: str) -> AsyncIterator[Any]:
        st = await self.drt.cp.subscribe(self.subject(event))
        return _decoding(st)


class Component:
    def __init__(self, ns: Namespace, name: str):
        self.namespace, self.name = ns, name
        self.drt = ns.drt

    @property
    def etcd_path(self) -> str:
        return f"{self.namespace.name}/components/{self.name}"

    @property
    def service_name(self) -> str:
        return slugify(f"{self.namespace.name}|{self.name}")

    def endpoint(self, name: str) -> "Endpoint":
        return Endpoint(self, name)

    async def create_service(self) -> "Component":
        await self.drt.server.start()
        return self

    async def create_service_with_custom_lease(self, ttl: float) -> Lease:
        await self.drt.server.start()
        return await self.drt.create_lease(ttl)

    def subject(self, event: str) -> str:
        return f"namespace.{self.namespace.name}.component.{self.name}.{event}"

    async def publish(self, event: str, payload: Any) -> None:
        await self.drt.cp.publish(self.subject(event), _enc(payload))

    async def subscribe(self, event: str) -> AsyncIterator[Any]:
        st = await self.drt.cp.subscribe(self.subject(event))
        return _decoding(st)

    async def scrape_stats(self, timeout: float = 0.3) -> list[dict]:
        """Collect every instance's endpoint stats (reference $SRV.STATS scrape,
        lib/runtime/src/service.rs:115)."""
        items = await self.drt.cp.get_prefix(self.etcd_path + "/")
        addrs = {}
        for _, v in items:
            info = json.loads(v)
            addrs[info["address"]] = info
        res = await asyncio.gather(*[scrape_stats(self.drt.pool, a, timeout) for a in addrs])
        out = []
        for (addr, info), st in zip(addrs.items(), res):
            if st is None:
                continue
            for path, data in st.items():
                if path.startswith(f"{self.namespace.name}/{self.name}/"):
                    out.append({"instance_id": info["lease_id"], "address": addr, "endpoint": path, "data": data})
        return out


@dataclass
class InstanceInfo:
    lease_id: int
    address: str
    namespace: str
    component: str
    endpoint: str
    path: str
    transport: str = "tcp"


class Endpoint:
    def __init__(self, component: Component, name: str):
        self.component, self.name = component, name
        self.drt = component.drt

    @property
    def path(self) -> str:
        return f"{self.component.namespace.name}/{self.component.name}/{self.name}"

    @property
    def etcd_prefix(self) -> str:
        return f"{self.component.etcd_path}/{self.name}:"

    def etcd_path_with_id(self, lease_id: int) -> str:
        return f"{self.etcd_prefix}{lease_id:x}"

    def subject_to(self, lease_id: int) -> str:
        return f"{self.component.service_name}.{slugify(self.name)}-{lease_id:x}"

    async def register(self, handler, lease: Lease | None = None, stats_handler=None) -> InstanceInfo:
        drt = self.drt
        await drt.server.start()
        drt.server.register(self.path, handler, stats_handler)
        lease = lease or drt.primary_lease
        lid = lease.id if lease else 0
        info = InstanceInfo(lid, drt.server.address, self.component.namespace.name, self.component.name, self.name,
                            self.path)
        ok = await drt.cp.create(self.etcd_path_with_id(lid), json.dumps(info.__dict__).encode(),
                                 lease=lid if lease else None)
        if not ok:
            raise RuntimeError(f"endpoint {self.path} already registered for lease {lid:x}")
        drt._served.append(self.path)
        if lease is not None:
            lease.on_lost.append(lambda: drt.server.unregister(self.path))
        return info

    async def serve_endpoint(self, handler, lease: Lease | None = None, stats_handler=None) -> None:
        """Register and serve until the runtime shuts down or the lease dies,
        then drain in-flight requests (graceful)."""
        lease = lease or self.drt.primary_lease
        await self.register(handler, lease, stats_handler)
        waiters = [asyncio.create_task(self.drt.shutdown_event.wait())]
        if lease is not None and lease is not self.drt.primary_lease:
            lost = asyncio.Event()
            lease.on_lost.append(lost.set)
            waiters.append(asyncio.create_task(lost.wait()))
        try:
            await asyncio.wait(waiters, return_when=asyncio.FIRST_COMPLETED)
        finally:
            for w in waiters:
                w.cancel()
            await self.drt.server.drain(self.path)

    async def client(self) -> "Client":
        c = Client(self)
        await c.start()
        return c

    def lease_id(self) -> int:
        return self.drt.primary_lease.id if self.drt.primary_lease else 0


class Client:
    """Watch-driven instance list + routing (random / round-robin / direct)."""

    def __init__(self, endpoint: Endpoint):
        self.endpoint = endpoint
        self.drt = endpoint.drt
        self.instances: dict[int, InstanceInfo] = {}
        self._rr = 0
        self._changed = asyncio.Event()
        self._task = None
        self._stream = None

    async def start(self) -> "Client":
        self._stream = await self.drt.cp.watch_prefix(self.endpoint.etcd_prefix)
        first = await self._stream.__anext__()
        for k, v, _ in first["items"]:
            self._add(v)
        self._task = asyncio.create_task(self._watch())
        return self

    def _add(self, v: bytes):
        d = json.loads(v)
        info = InstanceInfo(**d)
        self.instances[info.lease_id] = info
        self._changed.set()

    async def _watch(self):
        try:
            async for ev in self._stream:
                if ev["type"] == "put":
                    self._add(ev["value"])
                elif ev["type"] == "delete":
                    lid = int(ev["key"].rsplit(":", 1)[1], 16)
                    self.instances.pop(lid, None)
                    self._changed.set()
        except asyncio.CancelledError:
            pass

    async def close(self):
        if self._stream is not None:
            await self._stream.cancel()
        if self._task:
            self._task.cancel()

    def instance_ids(self) -> list[int]:
        return sorted(self.instances)

    async def wait_for_instances(self, timeout: float | None = None, n: int = 1) -> list[int]:
        async def _wait():
            while len(self.instances) < n:
                self._changed.clear()
                await self._changed.wait()

        await asyncio.wait_for(_wait(), timeout)
        return self.instance_ids()

    async def _call(self, lid: int, request: Any, context: Context | None) -> ResponseStream:
        info = self.instances.get(lid)
        if info is None:
            raise EndpointError(f"instance {lid:x} not found for {self.endpoint.path}")
        return await call_endpoint(self.drt.pool, info.address, self.endpoint.path, request, context)

    async def random(self, request: Any, context: Context | None = None) -> ResponseStream:
        ids = self.instance_ids()
        if not ids:
            raise EndpointError(f"no instances for {self.endpoint.path}")
        return await self._call(random.choice(ids), request, context)

    async def round_robin(self, request: Any, context: Context | None = None) -> ResponseStream:
        ids = self.instance_ids()
        if not ids:
            raise EndpointError(f"no instances for {self.endpoint.path}")
        lid = ids[self._rr % len(ids)]
        self._rr += 1
        return await self._call(lid, request, context)

    async def direct(self, request: Any, instance_id: int, context: Context | None = None) -> ResponseStream:
        return await self._call(instance_id, request, context)

    async def generate(self, request: Any, context: Context | None = None) -> ResponseStream:
        return await self.round_robin(request, context)


def _enc(payload: Any) -> bytes:
    if isinstance(payload, (bytes, bytearray)):
        return bytes(payload)
    if hasattr(payload, "model_dump_json"):
        return payload.model_dump_json().encode()
    return json.dumps(payload).encode()


async def _decoding(st):
    async for item in st:
        data = item["data"]
        try:
            yield json.loads(data)
        except Exception:
            yield data
