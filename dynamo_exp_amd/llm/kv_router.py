"""KV-cache-aware routing (reference lib/llm/src/kv_router*, examples/llm/components/kv_router.py).

Data flow:
  engine block pool --Stored/Removed--> KvEventPublisher --pub/sub "kv_events"--> KvIndexer (C++ radix tree)
  engine metrics    --ForwardPassMetrics--> KvMetricsPublisher --pub/sub "load_metrics"--> KvMetricsAggregator
  request tokens --> KvRouter.schedule: overlap scores x load --> worker id  (+ "kv-hit-rate" event)

Cost (reference scheduler.rs:290):
  logit = 2 * (overlap_blocks * block_size / isl) - kv_usage - active_slots / total_slots
Fixes vs reference: required_blocks uses ceil(isl / block_size);
an idle cluster is fine (no NoEndpoints at zero load); a logit of exactly 0 is
a valid choice; the optimistic load bump survives until the next metrics push.
Metrics are pushed by workers (every `interval`) instead of a 100 ms scrape,
but `KvMetricsAggregator.scrape()` can still pull the stats endpoint.
"""
from __future__ import annotations

import asyncio
import json
import logging
import random
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Callable

from .. import _native
from ..kv import hashing

log = logging.getLogger("dynamo_exp_amd.kv_router")

KV_EVENT_SUBJECT = "kv_events"
KV_METRICS_SUBJECT = "load_metrics"
KV_HIT_RATE_SUBJECT = "kv-hit-rate"


@dataclass
class ForwardPassMetrics:
    request_active_slots: int = 0
    request_total_slots: int = 1
    kv_active_blocks: int = 0
    kv_total_blocks: int = 1
    num_requests_waiting: int = 0
    gpu_cache_usage_perc: float = 0.0
    gpu_prefix_cache_hit_rate: float = 0.0


@dataclass
class KVHitRateEvent:
    worker_id: int
    isl_blocks: int
    overlap_blocks: int


# ================================================================ publishers
def _current_loop() -> asyncio.AbstractEventLoop | None:
    """The running loop, else the thread's set loop, else None (never creates one:
    after an asyncio.run() the main thread has no loop and get_event_loop raises)."""
    try:
        return asyncio.get_running_loop()
    except RuntimeError:
        pass
    try:
        return asyncio.get_event_loop_policy().get_event_loop()
    except RuntimeError:
        return None


class KvEventPublisher:
    """Publishes RouterEvent{worker_id, event{event_id, stored|removed}} for a
    worker; hooks onto LLMEngine.add_kv_event_listener (thread-safe)."""

    def __init__(self, component, worker_id: int, block_size: int, loop: asyncio.AbstractEventLoop | None = None):
        self.component = component
        self.worker_id = worker_id
        self.block_size = block_size
        self.loop = loop or _current_loop()
        self.event_id = 0

    def make_event(self, evs) -> dict:
        stored, removed = [], []
        parent = None
        for e in evs:
            if e.kind == "stored":
                if not stored:
                    parent = e.parent_hash
                stored.append({"block_hash": e.seq_hash, "tokens_hash": e.local_hash})
            else:
                removed.append(e.seq_hash)
        self.event_id += 1
        return {"worker_id": self.worker_id, "event_id": self.event_id, "stored_parent": parent, "stored": stored,
                "removed": removed}

    def on_engine_events(self, evs) -> None:
        # runs on the engine thread: group consecutive stores of one chain
        chains: list[list] = []
        for e in evs:
            if e.kind == "stored" and chains and chains[-1][0].kind == "stored" and \
                    e.parent_hash == chains[-1][-1].seq_hash:
                chains[-1].append(e)
            elif e.kind == "removed" and chains and chains[-1][0].kind == "removed":
                chains[-1].append(e)
            else:
                chains.append([e])
        for ch in chains:
            msg = self.make_event(ch)
            if self.loop is None:
                raise RuntimeError("KvEventPublisher: no event loop to publish on (pass loop=)")
            asyncio.run_coroutine_threadsafe(self.component.publish(KV_EVENT_SUBJECT, msg), self.loop)

    async def publish_stored(self, parent_hash: int | None, token_ids: list[int], block_hashes: list[int]) -> None:
        """C-ABI style publish (reference lib/bindings/c dynamo_kv_event_publish_stored): partial blocks dropped."""
        nb = len(token_ids) // self.block_size
        local = hashing.block_hashes(token_ids[: nb * self.block_size], self.block_size)
        self.event_id += 1
        await self.component.publish(KV_EVENT_SUBJECT, {
            "worker_id": self.worker_id, "event_id": self.event_id, "stored_parent": parent_hash,
            "stored": [{"block_hash": b, "tokens_hash": l} for b, l in zip(block_hashes[:nb], local)], "removed": []})

    async def publish_removed(self, block_hashes: list[int]) -> None:
        self.event_id += 1
        await self.component.publish(KV_EVENT_SUBJECT, {"worker_id": self.worker_id, "event_id": self.event_id,
                                                        "stored_parent": None, "stored": [],
                                                        "removed": list(block_hashes)})


class KvMetricsPublisher:
    def __init__(self, component, worker_id: int, metrics_fn: Callable[[], dict], interval: float = 0.1):
        self.component, self.worker_id = component, worker_id
        self.metrics_fn = metrics_fn
        self.interval = interval
        self._task = None
        self.last: dict = {}

    def stats_handler(self) -> dict:
        return self.metrics_fn()

    async def start(self) -> "KvMetricsPublisher":
        self._task = asyncio.create_task(self._loop())
        return self

    async def _loop(self):
        while True:
            try:
                m = self.metrics_fn()
                self.last = m
                await self.component.publish(KV_METRICS_SUBJECT, {"worker_id": self.worker_id, "metrics": m,
                                                                  "ts": time.time()})
            except asyncio.CancelledError:
                return
            except Exception:
                log.exception("metrics publish failed")
            await asyncio.sleep(self.interval)

    def stop(self):
        if self._task:
            self._task.cancel()


# ================================================================ indexer / aggregator
class KvIndexer:
    """Router-side global view of every worker's KV blocks (C++ radix tree).

    num_shards > 1: the sharded indexer (reference KvIndexerSharded,
    lib/llm/src/kv_router/indexer.rs:677-890) -- one actor thread per shard
    applying its workers' events, queries broadcast to every shard and merged.
    expiration_s: the frequency window (reference new_with_frequency,
    :202-275); `find_matches_scores` then also reports how often each matched
    depth was queried within the window."""

    def __init__(self, block_size: int, num_shards: int = 1, expiration_s: float | None = None):
        rt = _native.runtime()
        if rt is None:
            raise RuntimeError("_C_runtime required for the KV indexer")
        exp_ns = int(expiration_s * 1e9) if expiration_s else 0
        self.sharded = num_shards > 1
        self.tree = rt.ShardedRadixIndexer(num_shards, exp_ns) if self.sharded else rt.RadixIndexer(exp_ns)
        self.block_size = block_size
        self._task = None
        self.events = 0

    def apply(self, ev: dict) -> None:
        w = int(ev["worker_id"])
        if ev.get("stored"):
            self.tree.apply_stored(w, ev.get("stored_parent"), [b["block_hash"] for b in ev["stored"]],
                                   [b["tokens_hash"] for b in ev["stored"]])
        if ev.get("removed"):
            self.tree.apply_removed(w, list(ev["removed"]))
        self.events += 1

    def remove_worker(self, worker_id: int) -> None:
        self.tree.remove_worker(worker_id)

    def find_matches_for_request(self, tokens: list[int], early_exit: bool = False) -> dict[int, int]:
        if self.sharded:
            return self.find_matches_scores(hashing.block_hashes(list(tokens), self.block_size), early_exit)[0]
        return self.tree.find_matches_for_tokens(tokens, self.block_size, early_exit)

    def find_matches(self, local_hashes: list[int]) -> dict[int, int]:
        return self.find_matches_scores(local_hashes)[0]

    def find_matches_scores(self, local_hashes: list[int], early_exit: bool = False) -> tuple[dict[int, int], list[int]]:
        """(worker -> matched blocks, per-depth match frequencies in the window)."""
        scores, freq = self.tree.find_matches_freq(list(local_hashes), early_exit)
        return dict(scores), list(freq)

    def flush(self) -> None:
        """Sharded: wait until every event handed in so far is applied."""
        if self.sharded:
            self.tree.flush()

    async def start(self, component) -> "KvIndexer":
        sub = await component.subscribe(KV_EVENT_SUBJECT)

        async def loop():
            async for ev in sub:
                try:
                    self.apply(ev)
                except Exception:
                    log.exception("bad kv event")

        self._task = asyncio.create_task(loop())
        return self


class KvMetricsAggregator:
    def __init__(self, stale_after: float = 5.0):
        self.metrics: dict[int, tuple[float, ForwardPassMetrics]] = {}
        self.stale_after = stale_after
        self._task = None

    def update(self, worker_id: int, m: dict) -> None:
        self.metrics[int(worker_id)] = (time.monotonic(), ForwardPassMetrics(**{k: v for k, v in m.items()
                                                                              if k in ForwardPassMetrics.__dataclass_fields__}))

    def get_metrics(self) -> dict[int, ForwardPassMetrics]:
        now = time.monotonic()
        return {w: m for w, (t, m) in self.metrics.items() if now - t < self.stale_after}

    def remove(self, worker_id: int) -> None:
        self.metrics.pop(worker_id, None)

    def load_stats(self) -> tuple[float, float]:
        """(avg, std) of kv_active_blocks across workers (metrics component)."""
        vals = [m.kv_active_blocks for m in self.get_metrics().values()]
        if not vals:
            return 0.0, 0.0
        avg = sum(vals) / len(vals)
        return avg, (sum((v - avg) ** 2 for v in vals) / len(vals)) ** 0.5

    async def start(self, component) -> "KvMetricsAggregator":
        sub = await component.subscribe(KV_METRICS_SUBJECT)

        async def loop():
            async for msg in sub:
                try:
                    self.update(msg["worker_id"], msg["metrics"])
                except Exception:
                    log.exception("bad metrics message")

        self._task = asyncio.create_task(loop())
        return self

    async def scrape(self, component, timeout: float = 0.3) -> None:
        """Pull mode: read every instance's stats endpoint (reference 100 ms scrape)."""
        for s in await component.scrape_stats(timeout):
            d = s["data"]
            if isinstance(d, dict) and "kv_total_blocks" in d:
                self.update(s["instance_id"], d)


# ================================================================ selection
class DefaultWorkerSelector:
    def __init__(self, block_size: int, rng: random.Random | None = None):
        self.block_size = block_size
        self.rng = rng or random.Random()

    def select(self, workers: list[int], overlaps: dict[int, int], isl: int,
               metrics: dict[int, ForwardPassMetrics]) -> tuple[int, float]:
        best, best_logit = [], None
        isl = max(1, isl)
        # load term normalised by the busiest candidate, as the reference
        # scheduler does (lib/llm/src/kv_router/scheduler.rs:250-290); an
        # all-idle pool (max 0) is not an error here (§2.16), the term is 0
        max_active = max([(metrics.get(w) or ForwardPassMetrics()).request_active_slots for w in workers] or [0])
        for w in workers:
            m = metrics.get(w) or ForwardPassMetrics()
            score = overlaps.get(w, 0) * self.block_size / isl
            kv_use = m.kv_active_blocks / max(1, m.kv_total_blocks)
            load = m.request_active_slots / max_active if max_active > 0 else 0.0
            logit = 2.0 * score - kv_use - load
            if best_logit is None or logit > best_logit + 1e-9:
                best, best_logit = [w], logit
            elif abs(logit - best_logit) <= 1e-9:
                best.append(w)
        return self.rng.choice(best), best_logit


class KvRouter:
    """schedule(tokens) -> (worker_id, overlap_blocks); maintains optimistic load."""

    def __init__(self, component, block_size: int, selector=None, publish_hit_rate: bool = True,
                 indexer_shards: int = 1, expiration_s: float | None = None):
        self.component = component
        self.block_size = block_size
        self.indexer = KvIndexer(block_size, indexer_shards, expiration_s)
        self.metrics = KvMetricsAggregator()
        self.selector = selector or DefaultWorkerSelector(block_size)
        self.publish_hit_rate = publish_hit_rate
        self._bump: dict[int, int] = {}

    async def start(self) -> "KvRouter":
        await self.indexer.start(self.component)
        await self.metrics.start(self.component)
        return self

    def _metrics_with_bumps(self, workers: list[int] | None = None) -> dict[int, ForwardPassMetrics]:
        """Published metrics plus the requests routed since each worker's last
        refresh -- also for workers that have not published metrics yet."""
        ms = self.metrics.get_metrics()
        out = {}
        for w in set(ms) | set(workers or ()) | set(self._bump):
            m = ms.get(w) or ForwardPassMetrics()
            b = self._bump.get(w, 0)
            out[w] = ForwardPassMetrics(**{**asdict(m), "request_active_slots": m.request_active_slots + b})
        return out

    def schedule_sync(self, tokens: list[int], workers: list[int]) -> tuple[int, int]:
        if not workers:
            raise RuntimeError("no workers to route to")
        overlaps = self.indexer.find_matches_for_request(tokens)
        w, _ = self.selector.select(workers, overlaps, len(tokens), self._metrics_with_bumps(workers))
        self._bump[w] = self._bump.get(w, 0) + 1
        return w, overlaps.get(w, 0)

    async def schedule(self, tokens: list[int], workers: list[int]) -> tuple[int, int]:
        w, ov = self.schedule_sync(tokens, workers)
        if self.publish_hit_rate:
            isl_blocks = (len(tokens) + self.block_size - 1) // self.block_size
            try:
                await self.component.namespace.publish(KV_HIT_RATE_SUBJECT,
                                                       asdict(KVHitRateEvent(w, isl_blocks, ov)))
            except Exception:
                pass
        return w, ov

    def schedule_least_kv_load(self, workers: list[int]) -> tuple[int | None, float]:
        """`kv-load` routing (reference examples/llm/components/kv_router.py:
        226-245): the worker with the lowest KV-cache usage, random among
        ties.  (None, 0.0) when no metrics exist yet or every usage is zero,
        so the caller falls back to plain random routing as the reference does."""
        ms = self.metrics.get_metrics()
        load = {w: ms[w].kv_active_blocks / max(1, ms[w].kv_total_blocks) for w in workers if w in ms}
        if not load or not any(load.values()):
            return None, 0.0
        lo = min(load.values())
        w = self.selector.rng.choice([w for w, v in load.items() if v == lo])
        return w, lo

    def on_metrics_refresh(self, worker_id: int) -> None:
        self._bump.pop(worker_id, None)

    def release(self, worker_id: int) -> None:
        if self._bump.get(worker_id, 0) > 0:
            self._bump[worker_id] -= 1
