"""Reference-named Python API (`dynamo._core`,
lib/bindings/python/src/dynamo/_core.pyi) over this framework, so code
written against the reference's bindings maps one-to-one:

    from dynamo_exp_amd._core import DistributedRuntime, KvRouter, KvIndexer, EtcdKvCache, register_llm, ...

The classes are this framework's own implementations (native C++ radix
indexer / block hashing, in-tree control plane instead of etcd + NATS); this
module only provides the reference's names and call shapes where they differ.
"""
from __future__ import annotations

import asyncio
from dataclasses import dataclass, field

from .disagg.router import DisaggregatedRouter
from .llm.backend import Backend
from .llm.http_service import HttpService
from .llm.kv_router import ForwardPassMetrics, KvEventPublisher, KvMetricsPublisher
from .llm.kv_router import KvIndexer as _KvIndexer
from .llm.kv_router import KvMetricsAggregator as _KvMetricsAggregator
from .llm.kv_router import KvRouter as _KvRouter
from .llm.model_card import ModelDeploymentCard, attach
from .llm.preprocessor import OpenAIPreprocessor as OAIChatPreprocessor
from .llm.recorder import KvRecorder
from .runtime import Client, Component, Context, DistributedRuntime, Endpoint, Namespace
from .runtime import Lease as PyLease
from .runtime.transport import EndpointError as HttpError

__all__ = [
    "DistributedRuntime", "Namespace", "Component", "Endpoint", "Client", "PyLease", "Context", "EtcdClient",
    "EtcdKvCache", "KvRouter", "DisaggregatedRouter", "KvMetricsPublisher", "ModelDeploymentCard",
    "OAIChatPreprocessor", "Backend", "OverlapScores", "KvIndexer", "KvRecorder", "AggregatedMetrics",
    "KvMetricsAggregator", "KvEventPublisher", "HttpService", "HttpError", "ModelType", "register_llm",
    "ForwardPassMetrics",
]


class EtcdClient:
    """etcd-style KV API over the control plane (`drt.etcd_client()`)."""

    def __init__(self, drt: DistributedRuntime):
        self.drt = drt
        self.cp = drt.cp

    def primary_lease_id(self) -> int:
        return self.drt.primary_lease.id if self.drt.primary_lease else 0

    async def kv_create(self, key: str, value: bytes, lease_id: int | None = None) -> bool:
        return await self.cp.create(key, value, lease=lease_id)

    async def kv_create_or_validate(self, key: str, value: bytes, lease_id: int | None = None) -> bool:
        return await self.cp.create_or_validate(key, value, lease=lease_id)

    async def kv_put(self, key: str, value: bytes, lease_id: int | None = None) -> None:
        await self.cp.put(key, value, lease=lease_id)

    async def kv_get_prefix(self, prefix: str) -> list[dict]:
        return [{"key": k, "value": v} for k, v in await self.cp.get_prefix(prefix)]

    async def revoke_lease(self, lease_id: int) -> None:
        await self.cp.lease_revoke(lease_id)


class EtcdKvCache:
    """Watched prefix cache: `get` is a local lookup kept current by a watch
    (reference: Processor router mode / disagg thresholds live config)."""

    def __init__(self, client: EtcdClient, prefix: str):
        self.client, self.prefix = client, prefix
        self.data: dict[str, bytes] = {}
        self._task = None

    @staticmethod
    async def new(etcd_client: EtcdClient, prefix: str, initial_values: dict) -> "EtcdKvCache":
        c = EtcdKvCache(etcd_client, prefix)
        for k, v in initial_values.items():
            await etcd_client.kv_create(prefix + k, v.encode() if isinstance(v, str) else v)
        st = await etcd_client.cp.watch_prefix(prefix)
        snap = await st.__anext__()
        for k, v, _ in snap["items"]:
            c.data[k[len(prefix):]] = v

        async def loop():
            async for ev in st:
                key = ev["key"][len(prefix):]
                if ev["type"] == "put":
                    c.data[key] = ev["value"]
                else:
                    c.data.pop(key, None)

        c._task = asyncio.create_task(loop())
        return c

    async def get(self, key: str) -> bytes | None:
        return self.data.get(key)

    async def get_all(self) -> dict[str, bytes]:
        return dict(self.data)

    async def put(self, key: str, value: bytes | str, lease_id: int | None = None) -> None:
        await self.client.kv_put(self.prefix + key, value.encode() if isinstance(value, str) else value, lease_id)

    def close(self) -> None:
        if self._task:
            self._task.cancel()


@dataclass
class OverlapScores:
    scores: dict[int, int] = field(default_factory=dict)  # worker_id -> matched blocks
    frequencies: list[int] = field(default_factory=list)  # frequency window (reference OverlapScores)


@dataclass
class AggregatedMetrics:
    endpoints: list[dict] = field(default_factory=list)  # [{worker_id, **ForwardPassMetrics}]


def _start(coro):
    loop = asyncio.get_event_loop()
    return loop.create_task(coro)


class KvIndexer(_KvIndexer):
    """`KvIndexer(component, block_size)`: starts following `kv_events`."""

    def __init__(self, component: Component, block_size: int):
        super().__init__(block_size)
        self._start_task = _start(self.start(component))

    def find_matches_for_request(self, token_ids: list[int], lora_id: int = 0) -> OverlapScores:  # type: ignore[override]
        return OverlapScores(dict(super().find_matches_for_request(list(token_ids))))

    def block_size(self) -> int:  # type: ignore[override]
        return self.__dict__["block_size"]


class KvMetricsAggregator(_KvMetricsAggregator):
    def __init__(self, component: Component):
        super().__init__()
        self._start_task = _start(self.start(component))

    def get_metrics(self) -> AggregatedMetrics:  # type: ignore[override]
        from dataclasses import asdict

        return AggregatedMetrics([{"worker_id": w, **asdict(m)} for w, m in super().get_metrics().items()])


class KvRouter:
    """`KvRouter(drt, component, block_size)`; `await schedule(token_ids, lora_id)` -> worker id."""

    def __init__(self, drt: DistributedRuntime, component: Component, kv_block_size: int):
        self.drt, self.component = drt, component
        self.router = _KvRouter(component, kv_block_size)
        self._client = None
        self._ready = _start(self._init())

    async def _init(self):
        await self.router.start()
        self._client = await self.component.endpoint("generate").client()

    async def schedule(self, token_ids: list[int], lora_id: int = 0) -> int:
        await self._ready
        wid, _ = await self.router.schedule(list(token_ids), self._client.instance_ids())
        return wid


class ModelType:
    Chat = "chat"
    Completion = "completion"
    Backend = "backend"


async def register_llm(endpoint: Endpoint, path: str, model_type: str = ModelType.Backend,
                       router_mode: str = "round_robin") -> None:
    """Publish a model card + ModelEntry for `endpoint` (reference register_llm / LocalModel.attach)."""
    card = ModelDeploymentCard.load(path)
    await attach(endpoint.drt, endpoint, card, model_type, router_mode)
