"""Distributed runtime (reference layer L1 + Python helpers).

    from dynamo_exp_amd.runtime import DistributedRuntime, dynamo_worker, dynamo_endpoint

    @dynamo_worker()
    async def worker(runtime: DistributedRuntime):
        comp = runtime.namespace("demo").component("backend")
        await comp.create_service()
        await comp.endpoint("generate").serve_endpoint(handler)
"""
from __future__ import annotations

import asyncio
import functools
import inspect
import logging
import os
import signal
import sys

from .config import RuntimeConfig, WorkerConfig, is_truthy
from .context import Context
from .control_plane import BackgroundServer, ControlPlaneClient, ControlPlaneServer, SyncControlPlaneClient
from .distributed import Client, Component, DistributedRuntime, Endpoint, Lease, Namespace
from .logging_config import configure_logging
from .transport import EndpointError

__all__ = [
    "Context", "DistributedRuntime", "Namespace", "Component", "Endpoint", "Client", "Lease", "EndpointError",
    "ControlPlaneServer", "ControlPlaneClient", "SyncControlPlaneClient", "BackgroundServer", "dynamo_worker",
    "dynamo_endpoint", "configure_logging", "graceful_shutdown_timeout", "RuntimeConfig", "WorkerConfig",
    "is_truthy",
]

log = logging.getLogger("dynamo_exp_amd.runtime")


def graceful_shutdown_timeout() -> float:
    """DYN_WORKER_GRACEFUL_SHUTDOWN_TIMEOUT (reference worker.rs:51): 30 s."""
    return WorkerConfig.from_settings().graceful_shutdown_timeout


def dynamo_worker(static: bool = False, address: str | None = None):
    """Decorator for a worker main `async def main(runtime, *args)`.

    Creates the DistributedRuntime, traps SIGINT/SIGTERM into a graceful
    shutdown and exits with code 911 if draining exceeds the timeout
    (reference lib/runtime/src/worker.rs:99-150)."""

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            configure_logging()

            async def run():
                RuntimeConfig.from_settings().install(asyncio.get_running_loop())
                drt = await DistributedRuntime.create(address=address, is_static=static)
                loop = asyncio.get_running_loop()
                for sig in (signal.SIGINT, signal.SIGTERM):
                    try:
                        loop.add_signal_handler(sig, drt.shutdown)
                    except (NotImplementedError, RuntimeError):
                        pass
                main = asyncio.create_task(fn(drt, *args, **kwargs))
                stop = asyncio.create_task(drt.shutdown_event.wait())
                done, _ = await asyncio.wait([main, stop], return_when=asyncio.FIRST_COMPLETED)
                if main in done:
                    stop.cancel()
                    exc = main.exception()
                    await drt.close(graceful_shutdown_timeout())
                    if exc:
                        raise exc
                    return main.result()
                # shutdown requested: give the app the graceful window
                try:
                    await asyncio.wait_for(drt.close(graceful_shutdown_timeout()), graceful_shutdown_timeout() + 1)
                except asyncio.TimeoutError:
                    log.error("graceful shutdown timed out; exiting 911")
                    os._exit(911)
                main.cancel()

            return asyncio.run(run())

        return wrapper

    return deco


def dynamo_endpoint(request_model=None, response_model=None):
    """Validate requests/responses with pydantic models (reference
    lib/bindings/python/src/dynamo/runtime/__init__.py:60-95)."""

    def deco(fn):
        sig = inspect.signature(fn)
        nparams = len(sig.parameters)

        @functools.wraps(fn)
        async def wrapper(*args):
            args = list(args)
            idx = 1 if nparams >= 2 and list(sig.parameters)[0] == "self" else 0
            if request_model is not None and idx < len(args) and isinstance(args[idx], dict):
                args[idx] = request_model.model_validate(args[idx])
            async for item in fn(*args):
                if response_model is not None and isinstance(item, dict):
                    item = response_model.model_validate(item)
                yield item.model_dump() if hasattr(item, "model_dump") else item

        wrapper.__dynamo_endpoint__ = True
        wrapper.request_model = request_model
        wrapper.response_model = response_model
        return wrapper

    return deco
