"""Fake worker for router / metrics / planner tests without GPUs (reference
components/metrics/src/bin/mock_worker.rs).

  python -m dynamo_exp_amd.cli.mock_worker --namespace dynamo --component MyComponent

Serves `generate` (echoes each character of the request string, or each token
of `token_ids`) with a stats handler, and pushes random ForwardPassMetrics on
`load_metrics` every `--interval` seconds.
"""
from __future__ import annotations

import argparse
import asyncio
import random
from dataclasses import asdict

from ..llm.kv_router import ForwardPassMetrics, KvMetricsPublisher
from ..runtime import DistributedRuntime, configure_logging


def random_metrics(rng: random.Random) -> dict:
    total_slots, total_blocks = 100, 1000
    active_blocks = rng.randint(0, total_blocks)
    return asdict(ForwardPassMetrics(
        request_active_slots=rng.randint(0, total_slots), request_total_slots=total_slots,
        kv_active_blocks=active_blocks, kv_total_blocks=total_blocks, num_requests_waiting=rng.randint(0, 10),
        gpu_cache_usage_perc=active_blocks / total_blocks, gpu_prefix_cache_hit_rate=rng.random()))


async def echo(request, ctx=None):
    if isinstance(request, dict) and "token_ids" in request:
        for t in request["token_ids"]:
            yield {"token_ids": [t]}
    else:
        for ch in str(request):
            yield ch


async def serve(a, ready: asyncio.Event | None = None) -> None:
    drt = await DistributedRuntime.create(a.control_plane)
    comp = drt.namespace(a.namespace).component(a.component)
    await comp.create_service()
    rng = random.Random(a.seed)
    state = {"m": random_metrics(rng)}

    def metrics():
        state["m"] = random_metrics(rng)
        return state["m"]

    pub = await KvMetricsPublisher(comp, drt.primary_lease.id, metrics, a.interval).start()
    if ready is not None:
        ready.set()
    try:
        await comp.endpoint(a.endpoint).serve_endpoint(echo, stats_handler=lambda: state["m"])
    finally:
        pub.stop()


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(prog="mock_worker")
    ap.add_argument("--namespace", default="dynamo")
    ap.add_argument("--component", default="MyComponent")
    ap.add_argument("--endpoint", default="generate")
    ap.add_argument("--interval", type=float, default=0.5)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--control-plane", default=None)
    a = ap.parse_args(argv)
    configure_logging()
    asyncio.run(serve(a))


if __name__ == "__main__":
    main()
