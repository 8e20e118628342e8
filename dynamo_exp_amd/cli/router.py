"""Standalone KV-aware router service (reference components/router/src/main.rs:40-95).

  python -m dynamo_exp_amd.cli.router --namespace dynamo --component Worker [--block-size 64]
                                      [--selector module:Class] [--control-plane host:port]

Serves `{ns}/router/generate`: request `{"tokens": [...]}` (or a
PreprocessedRequest with `token_ids`), one response
`{"worker_id": id, "overlap_blocks": n, "prefix_hit_rate": f}`.  Indexes the
workers' `kv_events`, follows their `load_metrics`, and drops a worker from the
index when its endpoint registration disappears.  `--selector` plugs in a
custom WorkerSelector (`select(workers, overlaps, isl, metrics) -> (id, logit)`).
"""
from __future__ import annotations

import argparse
import asyncio
import importlib
import logging

from ..llm.kv_router import KvRouter
from ..runtime import DistributedRuntime, configure_logging

log = logging.getLogger("dynamo_exp_amd.router")


class RouterService:
    def __init__(self, drt, namespace: str, component: str, block_size: int, selector=None,
                 worker_endpoint: str = "generate", indexer_shards: int = 1):
        self.drt = drt
        self.indexer_shards = indexer_shards
        self.comp = drt.namespace(namespace).component(component)
        self.block_size = block_size
        self.selector = selector
        self.worker_endpoint = worker_endpoint
        self.kv: KvRouter | None = None
        self.client = None
        self._known: set[int] = set()

    async def start(self) -> "RouterService":
        self.kv = await KvRouter(self.comp, self.block_size, self.selector,
                                 indexer_shards=self.indexer_shards).start()
        self.client = await self.comp.endpoint(self.worker_endpoint).client()
        return self

    def _sync_workers(self) -> list[int]:
        live = set(self.client.instance_ids())
        for gone in self._known - live:
            self.kv.indexer.remove_worker(gone)
            self.kv.metrics.remove(gone)
        self._known = live
        return sorted(live)

    async def generate(self, request: dict, ctx=None):
        tokens = request.get("tokens") or request.get("token_ids") or []
        workers = self._sync_workers()
        if not workers:
            workers = await self.client.wait_for_instances(timeout=30)
        wid, overlap = await self.kv.schedule(list(tokens), workers)
        isl_blocks = max(1, (len(tokens) + self.block_size - 1) // self.block_size)
        yield {"worker_id": wid, "overlap_blocks": overlap, "prefix_hit_rate": overlap / isl_blocks}


def load_selector(spec: str | None, block_size: int):
    if not spec:
        return None
    mod, cls = spec.split(":")
    return getattr(importlib.import_module(mod), cls)(block_size)


async def serve(a) -> None:
    drt = await DistributedRuntime.create(a.control_plane)
    svc = await RouterService(drt, a.namespace, a.component, a.block_size,
                              load_selector(a.selector, a.block_size), a.worker_endpoint, a.indexer_shards).start()
    ep = drt.namespace(a.namespace).component("router").endpoint("generate")
    log.info("router serving %s for %s/%s", ep.path, a.namespace, a.component)
    await ep.serve_endpoint(svc.generate)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(prog="router")
    ap.add_argument("--namespace", default="dynamo")
    ap.add_argument("--component", default="Worker")
    ap.add_argument("--worker-endpoint", default="generate")
    ap.add_argument("--block-size", type=int, default=64)
    ap.add_argument("--selector", default=None)
    ap.add_argument("--indexer-shards", type=int, default=1,
                    help="KV indexer shards (actor threads; reference KvIndexerSharded)")
    ap.add_argument("--control-plane", default=None)
    a = ap.parse_args(argv)
    configure_logging()
    asyncio.run(serve(a))


if __name__ == "__main__":
    main()
