"""`@service`, `depends()`, `@dynamo_endpoint`, lifecycle hooks
(reference deploy/dynamo/sdk/src/dynamo/sdk/lib/{service,dependency,decorators}.py).

    @service(dynamo={"namespace": "inference"}, resources={"gpu": 1}, workers=2)
    class Worker:
        @dynamo_endpoint()
        async def generate(self, req: Request):
            yield ...

    @service(dynamo={"namespace": "inference"})
    class Frontend:
        worker = depends(Worker)
        @dynamo_endpoint(is_api=True)
        async def generate(self, req):
            async for r in self.worker.generate(req): yield r

`Frontend.link(Worker)` defines graph edges explicitly; `serve` starts every
service reachable from the entry service through links / dependencies.
"""
from __future__ import annotations

import inspect
import json
from dataclasses import asdict, dataclass, field
from typing import Any, AsyncIterator, Callable


@dataclass
class LeaseConfig:
    ttl: float = 1.0


@dataclass
class DynamoConfig:
    enabled: bool = True
    name: str | None = None
    namespace: str = "dynamo"
    custom_lease: LeaseConfig | None = None


class DynamoEndpoint:
    def __init__(self, fn: Callable, name: str | None = None, is_api: bool = False, request_model=None):
        self.fn = fn
        self.name = name or fn.__name__
        self.is_api = is_api
        params = list(inspect.signature(fn).parameters.values())
        self.request_model = request_model
        if self.request_model is None and len(params) >= 2:
            ann = params[1].annotation
            if inspect.isclass(ann) and hasattr(ann, "model_validate"):
                self.request_model = ann
        self.__name__ = self.name
        self.__doc__ = fn.__doc__
        self._with_ctx = len(params) >= 3

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self
        return _BoundEndpoint(self, obj)

    async def call(self, obj, request: Any, context=None) -> AsyncIterator[Any]:
        if isinstance(request, (str, bytes)) and self.request_model is not None:
            request = self.request_model.model_validate_json(request)
        elif isinstance(request, dict) and self.request_model is not None:
            request = self.request_model.model_validate(request)
        gen = self.fn(obj, request, context) if self._with_ctx else self.fn(obj, request)
        async for item in gen:
            yield item if type(item) is dict else (item.model_dump() if hasattr(item, "model_dump") else item)


class _BoundEndpoint:
    def __init__(self, ep: DynamoEndpoint, obj):
        self.ep, self.obj = ep, obj

    def __call__(self, request, context=None):
        return self.ep.call(self.obj, request, context)


def dynamo_endpoint(name: str | None = None, is_api: bool = False):
    def deco(fn):
        return DynamoEndpoint(fn, name, is_api)

    return deco


def async_on_start(fn):
    fn.__dynamo_on_start__ = True
    return fn


def async_on_shutdown(fn):
    fn.__dynamo_on_shutdown__ = True
    return fn


class DynamoService:
    def __init__(self, inner: type, dynamo: DynamoConfig, resources: dict, workers: int, app=None, envs=None):
        self.inner = inner
        self.name = inner.__name__
        self.dynamo = dynamo
        if self.dynamo.name is None:
            self.dynamo.name = self.name
        self.resources = dict(resources or {})
        self.workers = workers
        self.app = app
        self.envs = list(envs or [])
        self.endpoints: dict[str, DynamoEndpoint] = {}
        self.dependencies: dict[str, "Dependency"] = {}
        for attr in dir(inner):
            v = getattr(inner, attr, None)
            if isinstance(v, DynamoEndpoint):
                self.endpoints[v.name] = v
        for attr, v in list(vars(inner).items()):
            if isinstance(v, Dependency):
                self.dependencies[attr] = v
        self._links: list["DynamoService"] = []
        self._linked_explicitly = False

    def __repr__(self):
        return f"DynamoService({self.name})"

    def __call__(self, *a, **kw):
        return self.inner(*a, **kw)

    def link(self, other: "DynamoService") -> "DynamoService":
        """Declare an edge; when any link is declared, only linked deps are started."""
        self._links.append(other)
        self._linked_explicitly = True
        return other

    def dynamo_address(self) -> tuple[str, str]:
        return self.dynamo.namespace, self.dynamo.name

    def apply_overrides(self, cfg: dict) -> None:
        sa = (cfg.get(self.name) or {}).get("ServiceArgs") or {}
        if "workers" in sa:
            self.workers = int(sa["workers"])
        if "resources" in sa:
            self.resources.update(sa["resources"])
        for k, v in (sa.get("dynamo") or {}).items():
            if hasattr(self.dynamo, k):
                setattr(self.dynamo, k, LeaseConfig(**v) if k == "custom_lease" and isinstance(v, dict) else v)

    def graph(self) -> list["DynamoService"]:
        """All services reachable from this one (entry first)."""
        seen, order = set(), []

        def visit(s: "DynamoService"):
            if s.name in seen:
                return
            seen.add(s.name)
            order.append(s)
            deps = s._links if s._linked_explicitly else [d.target for d in s.dependencies.values()]
            for d in deps:
                visit(d)

        visit(self)
        return order

    def config_dict(self) -> dict:
        return {"name": self.name, "dynamo": asdict(self.dynamo), "resources": self.resources, "workers": self.workers,
                "endpoints": {k: {"is_api": v.is_api} for k, v in self.endpoints.items()},
                "dependencies": {k: v.target.name for k, v in self.dependencies.items()}}


def service(dynamo: dict | None = None, resources: dict | None = None, workers: int = 1, app=None, envs=None,
            **_ignored):
    def deco(cls):
        d = dict(dynamo or {})
        lease = d.pop("custom_lease", None)
        cfg = DynamoConfig(**{k: v for k, v in d.items() if k in DynamoConfig.__dataclass_fields__})
        if lease:
            cfg.custom_lease = lease if isinstance(lease, LeaseConfig) else LeaseConfig(**lease)
        return DynamoService(cls, cfg, resources or {}, workers, app, envs)

    return deco


class Dependency:
    """Class attribute; at runtime resolves to a DynamoClient proxy."""

    def __init__(self, target: DynamoService):
        self.target = target
        self.attr = None

    def __set_name__(self, owner, name):
        self.attr = name

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self
        clients = obj.__dict__.get("__dynamo_clients__", {})
        c = clients.get(self.attr)
        if c is None:
            raise RuntimeError(f"dependency {self.attr} used before the runtime connected it")
        return c


def depends(target: DynamoService) -> Dependency:
    return Dependency(target)


class DynamoClient:
    """`self.dep.<endpoint>(request)` -> async iterator over the remote stream."""

    def __init__(self, drt, svc: DynamoService):
        self.drt, self.svc = drt, svc
        self._clients: dict[str, Any] = {}
        self.mode = "round_robin"

    async def _client(self, ep: str):
        c = self._clients.get(ep)
        if c is None:
            ns, comp = self.svc.dynamo_address()
            c = await self.drt.namespace(ns).component(comp).endpoint(ep).client()
            await c.wait_for_instances(timeout=600)
            self._clients[ep] = c
        return c

    def __getattr__(self, ep: str):
        if ep.startswith("_"):
            raise AttributeError(ep)

        async def call(request, context=None, instance_id: int | None = None, mode: str | None = None):
            """`mode` (random | round_robin) overrides `self.mode` for this call
            only, so concurrent callers with different modes never race on
            the shared attribute."""
            c = await self._client(ep)
            if isinstance(request, str):
                try:
                    request = json.loads(request)
                except json.JSONDecodeError:
                    pass
            if hasattr(request, "model_dump"):
                request = request.model_dump()
            if instance_id is not None:
                stream = await c.direct(request, instance_id, context)
            elif (mode or self.mode) == "random":
                stream = await c.random(request, context)
            else:
                stream = await c.round_robin(request, context)
            async for item in stream:
                yield item

        return call

    async def client(self, ep: str = "generate"):
        return await self._client(ep)
