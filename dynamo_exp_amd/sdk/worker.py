"""Per-process entry for one service worker of a graph (reference
deploy/dynamo/sdk/src/dynamo/sdk/cli/serve_dynamo.py).

    python -m dynamo_exp_amd.sdk.worker <module:Service> --service-name <Name>

Creates the DistributedRuntime and the component (with the custom lease from
`dynamo.custom_lease`), instantiates the user class, connects `depends()`
clients, runs `@async_on_start` hooks, then serves every `@dynamo_endpoint`
concurrently; `is_api` endpoints are additionally exposed through the
service's FastAPI `app` (uvicorn) on its configured port.  The worker's lease
is recorded in the planner state file so the planner can drain it.
"""
from __future__ import annotations

import argparse
import asyncio
import importlib
import inspect
import json
import logging
import os
import sys

from fastapi import Request

from ..runtime import DistributedRuntime, configure_logging
from .config import ServiceConfig
from .service import DynamoClient, DynamoService
from .state import record_worker

log = logging.getLogger("dynamo_exp_amd.sdk.worker")


def load_service(target: str, name: str | None = None) -> DynamoService:
    mod_name, _, attr = target.partition(":")
    if mod_name.endswith(".py") or os.path.sep in mod_name:
        d = os.path.dirname(os.path.abspath(mod_name))
        sys.path.insert(0, d)
        mod_name = os.path.splitext(os.path.basename(mod_name))[0]
    else:
        sys.path.insert(0, os.getcwd())
    mod = importlib.import_module(mod_name)
    entry = getattr(mod, attr)
    if name is None or name == entry.name:
        return entry
    for s in entry.graph():
        if s.name == name:
            return s
    svc = getattr(mod, name, None)
    if isinstance(svc, DynamoService):
        return svc
    raise KeyError(f"service {name} not in graph {target}")


async def serve(svc: DynamoService, address: str | None = None) -> None:
    cfg = ServiceConfig.get_instance()
    svc.apply_overrides(cfg)
    drt = await DistributedRuntime.create(address)
    ns, comp_name = svc.dynamo_address()
    component = drt.namespace(ns).component(comp_name)
    await component.create_service()
    lease = drt.primary_lease
    if svc.dynamo.custom_lease is not None:
        lease = await component.create_service_with_custom_lease(svc.dynamo.custom_lease.ttl)
    obj = svc.inner.__new__(svc.inner)
    obj.__dict__["__dynamo_clients__"] = {a: DynamoClient(drt, d.target) for a, d in svc.dependencies.items()}
    obj.__dict__["__dynamo_runtime__"] = drt
    obj.__dict__["__dynamo_lease__"] = lease
    obj.__dict__["__dynamo_component__"] = component
    init = svc.inner.__init__
    if init is not object.__init__:
        init(obj)
    for name in dir(svc.inner):
        fn = getattr(obj, name, None)
        if callable(fn) and getattr(fn, "__dynamo_on_start__", False):
            r = fn()
            if inspect.isawaitable(r):
                await r
    record_worker(ns, svc.name, os.getpid(), lease.id if lease else 0)
    _tune_gc()
    tasks = []
    for ep_name, ep in svc.endpoints.items():
        endpoint = component.endpoint(ep_name)

        def make(ep=ep):
            def handler(req, ctx):  # the endpoint's own async generator: no extra hop per item
                return ep.call(obj, req, ctx)

            return handler

        tasks.append(asyncio.create_task(endpoint.serve_endpoint(make(), lease=lease)))
    api = [e for e in svc.endpoints.values() if e.is_api]
    if svc.app is not None and api:
        tasks.append(asyncio.create_task(_serve_api(svc, obj, api, cfg)))
    log.info("%s serving %s on %s (lease %x)", svc.name, list(svc.endpoints), drt.server.address,
             lease.id if lease else 0)
    stop = asyncio.create_task(drt.shutdown_event.wait())
    lease_lost = asyncio.Event()
    if lease is not None:
        lease.on_lost.append(lease_lost.set)
    lost = asyncio.create_task(lease_lost.wait())
    await asyncio.wait([stop, lost, *tasks], return_when=asyncio.FIRST_COMPLETED)
    if lost.done() and not stop.done():
        # lease revoked (planner scale-down): every endpoint stops accepting and
        # drains its in-flight requests (Endpoint.serve_endpoint), then the
        # shutdown hooks run (a prefill worker finishes what it dequeued)
        drained = asyncio.ensure_future(asyncio.gather(*tasks, return_exceptions=True))
        await asyncio.wait([drained, stop], timeout=float(os.environ.get("DYN_DRAIN_TIMEOUT_S", "120")),
                           return_when=asyncio.FIRST_COMPLETED)
    for name in dir(svc.inner):
        fn = getattr(obj, name, None)
        if callable(fn) and getattr(fn, "__dynamo_on_shutdown__", False):
            r = fn()
            if inspect.isawaitable(r):
                await r
    for t in tasks:
        t.cancel()
    await drt.close()


def _tune_gc() -> None:
    """Serving processes allocate a few short-lived objects per streamed token
    (frames, chunk dicts, generator hops) while holding thousands of long-lived
    ones (stream state, tokenizer tables): with the default thresholds the
    young-generation collector runs every ~700 allocations and keeps walking
    the survivors.  Freeze what start-up built and collect less often
    (DX_GC_THRESHOLD="gen0,gen1,gen2"; "default" keeps Python's)."""
    import gc

    spec = os.environ.get("DX_GC_THRESHOLD", "50000,20,100")
    if spec == "default":
        return
    gc.collect()
    gc.freeze()
    gc.set_threshold(*(int(x) for x in spec.split(",")))


async def _serve_api(svc: DynamoService, obj, api_eps, cfg) -> None:
    import uvicorn

    app = svc.app
    for ep in api_eps:
        app.add_api_route(f"/{ep.name}", _api_route(ep, obj), methods=["POST"])
    port = int((cfg.get(svc.name) or {}).get("port", 8000))
    server = uvicorn.Server(uvicorn.Config(app, host="0.0.0.0", port=port, log_level="warning"))
    await server.serve()


def _api_route(ep, obj):
    from fastapi.responses import StreamingResponse

    async def route(request: Request):
        body = await request.json()

        async def gen():
            async for item in ep.call(obj, body):
                yield (item if isinstance(item, str) else json.dumps(item)) + "\n"

        return StreamingResponse(gen(), media_type="text/plain")

    return route


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("target")
    ap.add_argument("--service-name", default=None)
    ap.add_argument("--control-plane", default=None)
    a, _ = ap.parse_known_args(argv)
    configure_logging()
    svc = load_service(a.target, a.service_name)
    # DX_PROFILE_DIR=<dir> [DX_PROFILE_SERVICES=Frontend,Processor]: cProfile
    # the service process, stats dumped at a clean exit (tools/frontend_scale.py)
    prof = None
    pdir = os.environ.get("DX_PROFILE_DIR")
    only = [s for s in os.environ.get("DX_PROFILE_SERVICES", "").split(",") if s]
    if pdir and (not only or svc.name in only):
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    try:
        asyncio.run(serve(svc, a.control_plane))
    finally:
        if prof is not None:
            prof.disable()
            os.makedirs(pdir, exist_ok=True)
            prof.dump_stats(os.path.join(pdir, f"{svc.name}.{os.getpid()}.prof"))


if __name__ == "__main__":
    main()
