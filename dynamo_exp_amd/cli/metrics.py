"""Prometheus exporter for worker load (reference components/metrics/src/lib.rs:125-430).

  python -m dynamo_exp_amd.cli.metrics --namespace dynamo --component Worker
                                       [--port 9091 | --push-gateway http://host:9091 --push-interval 2]

Follows the workers' pushed ForwardPassMetrics (`load_metrics`) -- or scrapes
their stats endpoints with `--scrape` -- and the namespace `kv-hit-rate`
events, and exports the reference's metric names:
  llm_kv_blocks_active / llm_kv_blocks_total / llm_requests_active_slots /
  llm_requests_total_slots / llm_kv_cache_usage_perc   {component, endpoint, worker_id}
  llm_load_avg / llm_load_std                           {component, endpoint}
  llm_kv_hit_rate_percent                               {component, endpoint, worker_id}
  llm_kv_hit_rate_isl_blocks / _overlap_blocks          counters
"""
from __future__ import annotations

import argparse
import asyncio
import logging

from prometheus_client import CollectorRegistry, Counter, Gauge, generate_latest, push_to_gateway, start_http_server

from ..llm.kv_router import KV_HIT_RATE_SUBJECT, KvMetricsAggregator
from ..runtime import DistributedRuntime, configure_logging

log = logging.getLogger("dynamo_exp_amd.metrics")


class PrometheusMetrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = r = registry or CollectorRegistry()
        lw = ["component", "endpoint", "worker_id"]
        self.kv_active = Gauge("llm_kv_blocks_active", "active KV blocks", lw, registry=r)
        self.kv_total = Gauge("llm_kv_blocks_total", "total KV blocks", lw, registry=r)
        self.req_active = Gauge("llm_requests_active_slots", "active request slots", lw, registry=r)
        self.req_total = Gauge("llm_requests_total_slots", "total request slots", lw, registry=r)
        self.cache_usage = Gauge("llm_kv_cache_usage_perc", "GPU KV cache usage", lw, registry=r)
        self.waiting = Gauge("llm_requests_waiting", "queued requests", lw, registry=r)
        self.load_avg = Gauge("llm_load_avg", "mean active KV blocks", ["component", "endpoint"], registry=r)
        self.load_std = Gauge("llm_load_std", "std of active KV blocks", ["component", "endpoint"], registry=r)
        self.hit_rate = Gauge("llm_kv_hit_rate_percent", "KV prefix hit rate of routed requests", lw, registry=r)
        self.isl_blocks = Counter("llm_kv_hit_rate_isl_blocks", "routed ISL blocks", lw, registry=r)
        self.overlap_blocks = Counter("llm_kv_hit_rate_overlap_blocks", "routed overlap blocks", lw, registry=r)
        self._hits: dict[int, list[int]] = {}

    def update(self, component: str, endpoint: str, agg: KvMetricsAggregator) -> None:
        for wid, m in agg.get_metrics().items():
            lab = (component, endpoint, str(wid))
            self.kv_active.labels(*lab).set(m.kv_active_blocks)
            self.kv_total.labels(*lab).set(m.kv_total_blocks)
            self.req_active.labels(*lab).set(m.request_active_slots)
            self.req_total.labels(*lab).set(m.request_total_slots)
            self.cache_usage.labels(*lab).set(m.gpu_cache_usage_perc)
            self.waiting.labels(*lab).set(m.num_requests_waiting)
        avg, std = agg.load_stats()
        self.load_avg.labels(component, endpoint).set(avg)
        self.load_std.labels(component, endpoint).set(std)

    def on_hit_rate(self, component: str, endpoint: str, ev: dict) -> None:
        wid = int(ev["worker_id"])
        lab = (component, endpoint, str(wid))
        self.isl_blocks.labels(*lab).inc(ev["isl_blocks"])
        self.overlap_blocks.labels(*lab).inc(ev["overlap_blocks"])
        tot = self._hits.setdefault(wid, [0, 0])
        tot[0] += ev["isl_blocks"]
        tot[1] += ev["overlap_blocks"]
        self.hit_rate.labels(*lab).set(100.0 * tot[1] / max(1, tot[0]))

    def exposition(self) -> bytes:
        return generate_latest(self.registry)


async def run(a, stop: asyncio.Event | None = None) -> PrometheusMetrics:
    drt = await DistributedRuntime.create(a.control_plane, is_static=True)
    ns = drt.namespace(a.namespace)
    comp = ns.component(a.component)
    agg = await KvMetricsAggregator().start(comp)
    pm = PrometheusMetrics()

    async def hits():
        async for ev in await ns.subscribe(KV_HIT_RATE_SUBJECT):
            pm.on_hit_rate(a.component, a.endpoint, ev)

    ht = asyncio.create_task(hits())
    if not a.push_gateway:
        start_http_server(a.port, addr=a.host, registry=pm.registry)
        log.info("metrics on http://%s:%d/metrics", a.host, a.port)
    stop = stop or asyncio.Event()
    while not stop.is_set():
        if a.scrape:
            await agg.scrape(comp)
        pm.update(a.component, a.endpoint, agg)
        if a.push_gateway:
            try:
                await asyncio.to_thread(push_to_gateway, a.push_gateway, "dynamo_metrics", pm.registry)
            except Exception as e:  # noqa: BLE001
                log.warning("push failed: %s", e)
        try:
            await asyncio.wait_for(stop.wait(), a.poll_interval)
        except asyncio.TimeoutError:
            pass
    ht.cancel()
    await drt.close(1)
    return pm


def arg_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="metrics")
    ap.add_argument("--namespace", default="dynamo")
    ap.add_argument("--component", default="Worker")
    ap.add_argument("--endpoint", default="load_metrics")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=9091)
    ap.add_argument("--push-gateway", default=None)
    ap.add_argument("--poll-interval", type=float, default=2.0)
    ap.add_argument("--scrape", action="store_true", help="pull stats endpoints instead of pushed metrics")
    ap.add_argument("--control-plane", default=None)
    return ap


def main(argv=None) -> None:
    a = arg_parser().parse_args(argv)
    configure_logging()
    asyncio.run(run(a))


if __name__ == "__main__":
    main()
