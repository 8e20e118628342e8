"""Load-based planner: grows/shrinks the prefill and decode pools on one node
(reference examples/llm/components/planner.py, docs/planner.md:37-78).

Every `metric_pulling_interval` (1 s) it samples
  * prefill queue load = queue depth / #prefill workers (control-plane queue)
  * decode KV load     = mean gpu_cache_usage_perc over decode workers (pushed ForwardPassMetrics)
and every `adjustment_interval` (30 s) scales by at most +-1 worker per pool:
  scale down prefill  if queue load < 0.2 and #P > min
  scale down decode   if kv load < 0.5 and #D > min and no grace period
  scale up prefill    if queue load > 0.5, trend-extrapolated load (3 periods) still > 0.5, GPU budget allows
  scale up decode     if kv load > 0.9 and GPU budget allows (then 3-interval grace period)
Metrics and decisions go to a JSONL log (TensorBoard in the reference).
`--no-operation` observes only.

`--policy utilization` (ours) adds the signal the queue-depth rule lacks: the
prefill workers' device-busy fraction (their `mock` endpoint), because an
empty prefill queue only says the pool keeps up, not that it could lose a
worker.  Prefill scales down only when the remaining workers would stay under
`prefill_util_target` busy, scales up on a long queue OR a saturated pool (and
by two workers when the backlog is several intervals deep); decode scales down
only when the remaining workers would stay under the scale-up threshold.  A
pool that shrinks into the next peak and then queues for the adjustment
intervals it takes to grow back is what made the reference rule oscillate
under the 15-60 req/s trace (profiles/r3_planner_bench_x3_*.json).

`--policy rate` (ours, predictive) sizes the prefill pool from the prompt
ARRIVAL rate instead of reacting to a queue that already exists: every
sample estimates the arrival rate into the prefill queue (prompts the
workers dequeued + the queue's growth, per second; workers report their
`dequeued` counters on `mock`) and the per-worker service capacity (dequeue
rate over device-busy worker-seconds); at each adjustment a linear fit over
the last `rate_window_s` forecasts the arrival rate one adjustment interval +
worker start-up ahead, and the pool is set to ceil((forecast + backlog /
horizon) / (capacity x rate_util_target)) workers -- several at once when a
ramp needs them -- and shrinks by one only when the forecast fits the smaller
pool for two adjustments in a row and no prefill worker was added in the last
`prefill_scale_down_delay_s`.  Decode scales as in `utilization`, or, with
`decode_streams_target` S > 0, to ceil(forecast streams / S) workers: the
active streams (the decode workers' request_active_slots) scaled by the
arrival-rate forecast's ahead / now ratio -- the decode step time grows with
the streams a worker batches, so S pins the inter-token latency (S = 40 on the
3.5x-slowed sim: ITL ~32 ms; tools/planner_oracle.py: the clairvoyant optimum
keeps 21-46 streams per decode worker across the trace), several workers at
once on a ramp, one at a time (two agreeing intervals, no add in the last
`prefill_scale_down_delay_s`) on the way down.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import subprocess
import sys
import time
from dataclasses import dataclass, field

from ..llm.kv_router import KvMetricsAggregator
from ..runtime import DistributedRuntime, configure_logging
from .connector import LocalConnector

log = logging.getLogger("dynamo_exp_amd.planner")

NEW_DECODE_WORKER_GRACE_PERIOD = 3
WORKER_START_TIMEOUT_S = 300.0  # a requested worker not registered by then no longer counts
NEW_PREFILL_WORKER_QUEUE_BUFFER_PERIOD = 3


@dataclass
class PlannerConfig:
    namespace: str = "dynamo"
    decode_component: str = "Worker"
    prefill_component: str = "PrefillWorker"
    prefill_queue: str = "prefill_queue"
    metric_pulling_interval: float = 1.0
    adjustment_interval: float = 30.0
    prefill_queue_scale_up_threshold: float = 0.5
    prefill_queue_scale_down_threshold: float = 0.2
    decode_kv_scale_up_threshold: float = 0.9
    decode_kv_scale_down_threshold: float = 0.5
    # decode load signal: "kv" = mean KV-cache usage (reference); "kv_slots" =
    # mean of max(KV usage, active request slots / slots) -- on a 288 GB MI355X
    # an 8B decode engine runs out of request slots (max_num_seqs) long before
    # its KV cache fills (~2M tokens), so KV usage alone never signals load
    decode_load_metric: str = "kv_slots"
    min_endpoint: int = 1
    max_gpu_budget: int = 8
    prefill_engine_num_gpu: int = 1
    decode_engine_num_gpu: int = 1
    no_operation: bool = False
    log_dir: str | None = None
    policy: str = "reference"  # "reference" | "utilization" | "rate"
    prefill_util_target: float = 0.75
    prefill_util_scale_up_threshold: float = 0.92
    # rate policy
    rate_window_s: float = 30.0  # arrival-rate fit window
    # provision the forecast at this fraction of a worker's measured capacity (1.0: -20 % latency for +1.7 %
    # GPU-s vs static 2P2D; 0.85: +8.4 % GPU-s for the same latency -- profiles/r5_planner_rate_summary.txt)
    rate_util_target: float = 1.0
    worker_startup_s: float = 10.0  # from an add to a serving worker (forecast horizon = interval + this)
    # utilization / rate policies: no prefill scale-down this long after a prefill scale-up.  Right after an
    # add the queue is drained and the busy fraction / capacity estimate come from a handful of samples; acting
    # on them removed the new worker 10-15 s later (CPU dry runs of tools/planner_gpu_check.py, both policies)
    prefill_scale_down_delay_s: float = 30.0
    prefill_worker_capacity: float = 0.0  # prompts/s per prefill worker; 0 = estimated online
    decode_streams_target: float = 0.0  # rate policy: active streams per decode worker (0 = the KV-load rule)
    rate_shrink_step: int = 1  # rate policy: workers removed per agreed scale-down (0 = down to the target at once)


@dataclass
class PlannerState:
    n_prefill: int
    n_decode: int
    prefill_queue_load: list[float] = field(default_factory=list)
    kv_load: list[float] = field(default_factory=list)
    decode_grace: int = 0
    prefill_util: list[float] = field(default_factory=list)  # mean busy fraction of the prefill pool per sample
    # rate policy (kept across adjustments by the Planner): (t, arrival prompts/s) samples, the
    # capacity estimate (prompts/s per busy worker-second), the current queue depth
    arrivals: list = field(default_factory=list)
    capacity: float = 0.0
    queue: int = 0
    shrink_votes: int = 0
    since_prefill_add: float = float("inf")  # seconds since the last prefill scale-up
    decode_streams: list[float] = field(default_factory=list)  # active streams over all decode workers per sample
    decode_shrink_votes: int = 0
    since_decode_add: float = float("inf")


def decode_load(m, metric: str = "kv_slots") -> float:
    """One decode worker's load from its ForwardPassMetrics."""
    kv = float(m.gpu_cache_usage_perc)
    if metric == "kv":
        return kv
    slots = m.request_active_slots / max(1, m.request_total_slots)
    return max(kv, slots)


def decide(cfg: PlannerConfig, st: PlannerState) -> list[tuple[str, str]]:
    """Pure policy: returns [(action, component)] with action in {add, remove}."""
    if cfg.policy == "utilization":
        return decide_utilization(cfg, st)
    if cfg.policy == "rate":
        return decide_rate(cfg, st)
    acts = []
    gpus = st.n_prefill * cfg.prefill_engine_num_gpu + st.n_decode * cfg.decode_engine_num_gpu
    q = sum(st.prefill_queue_load) / len(st.prefill_queue_load) if st.prefill_queue_load else 0.0
    kv = sum(st.kv_load) / len(st.kv_load) if st.kv_load else 0.0
    if q < cfg.prefill_queue_scale_down_threshold and st.n_prefill > cfg.min_endpoint:
        acts.append(("remove", cfg.prefill_component))
        gpus -= cfg.prefill_engine_num_gpu
    if kv < cfg.decode_kv_scale_down_threshold and st.n_decode > cfg.min_endpoint and st.decode_grace <= 0:
        acts.append(("remove", cfg.decode_component))
        gpus -= cfg.decode_engine_num_gpu
    if q > cfg.prefill_queue_scale_up_threshold and gpus + cfg.prefill_engine_num_gpu <= cfg.max_gpu_budget:
        trend = st.prefill_queue_load[-1] - st.prefill_queue_load[0] if st.prefill_queue_load else 0.0
        predicted = (st.prefill_queue_load[-1] if st.prefill_queue_load else 0.0) + \
            trend * NEW_PREFILL_WORKER_QUEUE_BUFFER_PERIOD
        if predicted > cfg.prefill_queue_scale_up_threshold:
            acts.append(("add", cfg.prefill_component))
            gpus += cfg.prefill_engine_num_gpu
    if kv > cfg.decode_kv_scale_up_threshold and gpus + cfg.decode_engine_num_gpu <= cfg.max_gpu_budget:
        acts.append(("add", cfg.decode_component))
    return acts


def decide_utilization(cfg: PlannerConfig, st: PlannerState) -> list[tuple[str, str]]:
    """The `utilization` policy (module docstring)."""
    acts = []
    gpus = st.n_prefill * cfg.prefill_engine_num_gpu + st.n_decode * cfg.decode_engine_num_gpu
    ql = st.prefill_queue_load
    q = sum(ql) / len(ql) if ql else 0.0
    q_max = max(ql) if ql else 0.0
    util = sum(st.prefill_util) / len(st.prefill_util) if st.prefill_util else 0.0
    kv = sum(st.kv_load) / len(st.kv_load) if st.kv_load else 0.0
    kv_max = max(st.kv_load) if st.kv_load else 0.0
    n_p, n_d = st.n_prefill, st.n_decode
    # prefill
    if q > cfg.prefill_queue_scale_up_threshold or util > cfg.prefill_util_scale_up_threshold:
        trend = ql[-1] - ql[0] if ql else 0.0
        backlog = (ql[-1] if ql else 0.0) + max(0.0, trend) * NEW_PREFILL_WORKER_QUEUE_BUFFER_PERIOD
        want = 2 if backlog > 4 * cfg.prefill_queue_scale_up_threshold * max(1, n_p) else 1
        for _ in range(want):
            if gpus + cfg.prefill_engine_num_gpu <= cfg.max_gpu_budget:
                acts.append(("add", cfg.prefill_component))
                gpus += cfg.prefill_engine_num_gpu
    elif (n_p > cfg.min_endpoint and q_max < cfg.prefill_queue_scale_down_threshold
          and st.since_prefill_add >= cfg.prefill_scale_down_delay_s
          and util * n_p / (n_p - 1) < cfg.prefill_util_target):
        acts.append(("remove", cfg.prefill_component))
        gpus -= cfg.prefill_engine_num_gpu
    # decode
    if kv > cfg.decode_kv_scale_up_threshold and gpus + cfg.decode_engine_num_gpu <= cfg.max_gpu_budget:
        acts.append(("add", cfg.decode_component))
    elif (n_d > cfg.min_endpoint and st.decode_grace <= 0 and kv < cfg.decode_kv_scale_down_threshold
          and kv_max * n_d / (n_d - 1) < cfg.decode_kv_scale_up_threshold):
        acts.append(("remove", cfg.decode_component))
    return acts


def forecast(samples: list, window: float, horizon: float) -> tuple[float, float]:
    """(rate now, rate `horizon` s ahead) from a least-squares line over the
    (t, rate) samples of the last `window` seconds."""
    if not samples:
        return 0.0, 0.0
    t_last = samples[-1][0]
    pts = [(t, r) for t, r in samples if t >= t_last - window]
    n = len(pts)
    if n < 3:
        r = sum(r for _, r in pts) / n
        return r, r
    mt = sum(t for t, _ in pts) / n
    mr = sum(r for _, r in pts) / n
    var = sum((t - mt) ** 2 for t, _ in pts)
    slope = sum((t - mt) * (r - mr) for t, r in pts) / var if var > 0 else 0.0
    now = mr + slope * (t_last - mt)
    return max(0.0, now), max(0.0, now + slope * horizon)


def decide_rate(cfg: PlannerConfig, st: PlannerState) -> list[tuple[str, str]]:
    """The `rate` policy (module docstring)."""
    import math

    cap = cfg.prefill_worker_capacity or st.capacity
    if cap <= 0:  # no capacity estimate yet (pool never busy): the reactive policy
        return decide_utilization(cfg, st)
    acts = []
    gpus = st.n_prefill * cfg.prefill_engine_num_gpu + st.n_decode * cfg.decode_engine_num_gpu
    horizon = cfg.adjustment_interval + cfg.worker_startup_s
    now, ahead = forecast(st.arrivals, cfg.rate_window_s, horizon)
    per = cap * cfg.rate_util_target
    need = (max(now, ahead) + st.queue / horizon) / per
    budget_p = (cfg.max_gpu_budget - st.n_decode * cfg.decode_engine_num_gpu) // cfg.prefill_engine_num_gpu
    target = max(cfg.min_endpoint, min(budget_p, math.ceil(need - 1e-9)))
    n_p = st.n_prefill
    if target > n_p:
        st.shrink_votes = 0
        for _ in range(target - n_p):
            if gpus + cfg.prefill_engine_num_gpu <= cfg.max_gpu_budget:
                acts.append(("add", cfg.prefill_component))
                gpus += cfg.prefill_engine_num_gpu
    elif (n_p > cfg.min_endpoint and st.queue <= n_p and st.since_prefill_add >= cfg.prefill_scale_down_delay_s
          and (max(now, ahead) + st.queue / horizon) / per <= n_p - 1):
        st.shrink_votes += 1
        if st.shrink_votes >= 2:  # two intervals in a row: not a dip inside a peak
            # down to the forecast's pool in one go (or one at a time: rate_shrink_step = 1)
            n_rm = n_p - target if cfg.rate_shrink_step == 0 else min(cfg.rate_shrink_step, n_p - target)
            for _ in range(max(1, n_rm)):
                acts.append(("remove", cfg.prefill_component))
                gpus -= cfg.prefill_engine_num_gpu
            st.shrink_votes = 0
    else:
        st.shrink_votes = 0
    n_d = st.n_decode
    if cfg.decode_streams_target > 0 and st.decode_streams:
        return acts + _decode_by_streams(cfg, st, now, ahead, gpus)
    kv = sum(st.kv_load) / len(st.kv_load) if st.kv_load else 0.0
    kv_max = max(st.kv_load) if st.kv_load else 0.0
    if kv > cfg.decode_kv_scale_up_threshold and gpus + cfg.decode_engine_num_gpu <= cfg.max_gpu_budget:
        acts.append(("add", cfg.decode_component))
    elif (n_d > cfg.min_endpoint and st.decode_grace <= 0 and kv < cfg.decode_kv_scale_down_threshold
          and kv_max * n_d / (n_d - 1) < cfg.decode_kv_scale_up_threshold):
        acts.append(("remove", cfg.decode_component))
    return acts


def _decode_by_streams(cfg: PlannerConfig, st: PlannerState, now: float, ahead: float, gpus: int) -> list:
    """The rate policy's decode rule with a streams-per-worker target (module docstring)."""
    import math

    recent = st.decode_streams[-max(1, len(st.decode_streams) // 3):]  # the last third of the interval
    streams = sum(recent) / len(recent)
    growth = ahead / now if now > 0 else 1.0
    want = streams * max(1.0, growth)
    budget_d = (cfg.max_gpu_budget - (gpus - st.n_decode * cfg.decode_engine_num_gpu)) // cfg.decode_engine_num_gpu
    target = max(cfg.min_endpoint, min(budget_d, math.ceil(want / cfg.decode_streams_target - 1e-9)))
    n_d = st.n_decode
    acts = []
    if target > n_d:
        st.decode_shrink_votes = 0
        for _ in range(target - n_d):
            acts.append(("add", cfg.decode_component))
    elif (n_d > cfg.min_endpoint and st.since_decode_add >= cfg.prefill_scale_down_delay_s
          and streams * growth / (n_d - 1) <= cfg.decode_streams_target):
        st.decode_shrink_votes += 1
        if st.decode_shrink_votes >= 2:
            n_rm = n_d - target if cfg.rate_shrink_step == 0 else min(cfg.rate_shrink_step, n_d - target)
            for _ in range(max(1, n_rm)):
                acts.append(("remove", cfg.decode_component))
            st.decode_shrink_votes = 0
    else:
        st.decode_shrink_votes = 0
    return acts


class Planner:
    def __init__(self, drt: DistributedRuntime, cfg: PlannerConfig, connector: LocalConnector | None = None):
        self.drt, self.cfg = drt, cfg
        self.connector = connector or LocalConnector(cfg.namespace, drt)
        self.ns = drt.namespace(cfg.namespace)
        self.metrics = KvMetricsAggregator()
        self.state = PlannerState(0, 0)
        self.log_path = None
        self.t0 = time.time()
        self.p_client = self.d_client = None
        # rate policy: last (t, queue, {instance: dequeued}) sample, arrival history, capacity estimate
        self._last = None
        self._base: dict = {}  # instance -> (t, dequeued) of its last answer
        self._arrivals: list = []
        self._cap_num = self._cap_den = 0.0
        self._shrink_votes = 0
        self._decode_shrink_votes = 0
        self._last_prefill_add = None
        self._last_decode_add = None
        self._expect: dict[str, tuple[int, float]] = {}  # component -> (workers expected, when requested)
        self._registered = (0, 0)

    async def start(self) -> "Planner":
        await self.metrics.start(self.ns.component(self.cfg.decode_component))
        self.d_client = await self.ns.component(self.cfg.decode_component).endpoint("generate").client()
        self.p_client = await self.ns.component(self.cfg.prefill_component).endpoint("mock").client()
        d = self.cfg.log_dir or os.path.join("logs", time.strftime("%m%d_%H%M%S"))
        os.makedirs(d, exist_ok=True)
        self.log_path = os.path.join(d, "planner.jsonl")
        return self

    def _log(self, **kw):
        kw["t"] = round(time.time() - self.t0, 2)
        with open(self.log_path, "a") as f:
            f.write(json.dumps(kw) + "\n")

    def workers(self) -> tuple[int, int]:
        return len(self.p_client.instance_ids()), len(self.d_client.instance_ids())

    async def collect_metrics(self) -> None:
        n_p, n_d = self.workers()
        qsize = await self.drt.cp.q_size(self.cfg.prefill_queue)
        qload = qsize / max(1, n_p)
        ms = self.metrics.get_metrics()
        kv = sum(decode_load(m, self.cfg.decode_load_metric) for m in ms.values()) / len(ms) if ms else 0.0
        self.state.decode_streams.append(float(sum(m.request_active_slots for m in ms.values())))
        util, counts = await self.prefill_utilization(with_counts=True)
        self.state.prefill_queue_load.append(qload)
        self.state.kv_load.append(kv)
        if util is not None:
            self.state.prefill_util.append(util)
        arrival = self._arrival_sample(time.time(), qsize, counts, util, n_p)
        self._log(kind="metrics", prefill_queue=qsize, prefill_queue_load=qload, kv_load=kv, n_prefill=n_p,
                  n_decode=n_d, prefill_util=util, arrival_rate=arrival)

    def _arrival_sample(self, now: float, qsize: int, counts: dict, util, n_p: int) -> float | None:
        """Prompts/s entering the prefill queue since the last sample (dequeued
        by the workers + the queue's growth), and the capacity estimate
        (dequeued per busy worker-second).

        Each worker's `dequeued` counter is cumulative, so it is differenced
        against that worker's OWN last answer: a worker that misses
        a sample (its `mock` answer timed out while busy) keeps its baseline
        and is counted at its next answer, as a rate over the time since its
        last one; a worker seen for the first time only sets its baseline --
        its lifetime count is never taken as one interval's arrivals."""
        last, self._last = self._last, (now, qsize, counts)
        if last is None:
            for i, v in counts.items():
                self._base[i] = (now, v)
            return None
        t0, q0, _ = last
        dt = now - t0
        if dt <= 0:
            return None
        deq_rate = 0.0  # prompts/s dequeued, per worker over its own interval
        deq = 0
        complete = bool(counts)  # every known worker answered, none is new: a clean capacity sample
        for i, v in counts.items():
            b = self._base.get(i)
            self._base[i] = (now, v)
            if b is None:
                complete = False
                continue
            d = max(0, v - b[1])
            deq += d
            deq_rate += d / max(now - b[0], 1e-6)
        if any(i not in counts and tb >= t0 for i, (tb, _) in self._base.items()):
            complete = False  # a worker that answered last time is missing now
        rate = max(0.0, deq_rate + (qsize - q0) / dt)
        self._arrivals.append((now, rate))
        if len(self._arrivals) > 600:
            del self._arrivals[:-600]
        busy = (util or 0.0) * n_p * dt
        if complete and util is not None and util > 0.5 and busy > 0:  # a mostly busy pool: its rate is its capacity
            self._cap_num = 0.9 * self._cap_num + deq
            self._cap_den = 0.9 * self._cap_den + busy
        return round(rate, 3)

    async def prefill_utilization(self, with_counts: bool = False):
        """Mean device-busy fraction of the prefill workers (each worker's
        `mock` endpoint); None when no worker answered.  with_counts: also
        {instance: prompts dequeued so far}."""

        async def one(iid):
            try:
                async def first():
                    async for r in await self.p_client.direct({}, iid):
                        return r

                r = await asyncio.wait_for(first(), 0.5)
                return r if isinstance(r, dict) else None
            except Exception:  # noqa: BLE001  (a worker going away mid-sample)
                return None

        ids = self.p_client.instance_ids()
        rs = await asyncio.gather(*(one(i) for i in ids))
        vals = [float(r["busy"]) for r in rs if r is not None and r.get("busy") is not None]
        util = sum(vals) / len(vals) if vals else None
        if not with_counts:
            return util
        counts = {i: int(r["dequeued"]) for i, r in zip(ids, rs) if r is not None and r.get("dequeued") is not None}
        return util, counts

    def _effective(self, comp: str, registered: int) -> int:
        """Workers of `comp` counting requested-but-not-yet-registered ones: an
        engine takes tens of seconds to start, and without this the next
        adjustment sees the old count and adds again (round-5 GPU check: two
        prefill workers added 5 s apart for one overload, past the budget)."""
        want, t = self._expect.get(comp, (0, 0.0))
        if time.time() - t > WORKER_START_TIMEOUT_S or registered >= want:
            self._expect.pop(comp, None)
            return registered
        return want

    async def make_adjustments(self) -> list:
        n_p, n_d = self.workers()
        if (n_p, n_d) != self._registered:
            log.info("workers changed during the interval; skipping adjustment")
            acts = []
        else:
            self._prime_rate_state()
            acts = decide(self.cfg, self.state)
        self._log(kind="adjust", actions=acts, n_prefill=n_p, n_decode=n_d,
                  **({"capacity": round(self.state.capacity, 3)} if self.cfg.policy == "rate" else {}))
        if not self.cfg.no_operation:
            eff = {self.cfg.prefill_component: self.state.n_prefill, self.cfg.decode_component: self.state.n_decode}
            for act, comp in acts:
                ok = await (self.connector.add_component(comp) if act == "add"
                            else self.connector.remove_component(comp))
                log.info("%s %s -> %s", act, comp, ok)
                if ok and act == "add":
                    eff[comp] = eff.get(comp, 0) + 1
                    self._expect[comp] = (eff[comp], time.time())
                    if comp == self.cfg.prefill_component:
                        self._last_prefill_add = time.time()
                    if comp == self.cfg.decode_component:
                        self.state.decode_grace = NEW_DECODE_WORKER_GRACE_PERIOD
                        self._last_decode_add = time.time()
                elif ok:
                    eff[comp] = max(0, eff.get(comp, 0) - 1)
                    if comp in self._expect:
                        self._expect[comp] = (eff[comp], self._expect[comp][1])
        if self.state.decode_grace > 0:
            self.state.decode_grace -= 1
        self._refresh_state()
        return acts

    def _refresh_state(self) -> None:
        n_p, n_d = self.workers()
        self._registered = (n_p, n_d)
        self._shrink_votes = self.state.shrink_votes
        self._decode_shrink_votes = self.state.decode_shrink_votes
        self.state = PlannerState(self._effective(self.cfg.prefill_component, n_p),
                                  self._effective(self.cfg.decode_component, n_d), decode_grace=self.state.decode_grace)
        self._prime_rate_state()

    def _prime_rate_state(self) -> None:
        st = self.state
        st.arrivals = self._arrivals
        st.capacity = self._cap_num / self._cap_den if self._cap_den > 0 else 0.0
        st.queue = self._last[1] if self._last else 0
        st.shrink_votes = self._shrink_votes
        st.since_prefill_add = time.time() - self._last_prefill_add if self._last_prefill_add else float("inf")
        st.decode_shrink_votes = self._decode_shrink_votes
        st.since_decode_add = time.time() - self._last_decode_add if self._last_decode_add else float("inf")

    async def run(self, duration: float | None = None) -> None:
        self._refresh_state()
        end = time.time() + duration if duration else None
        last_adjust = time.time()
        while end is None or time.time() < end:
            await self.collect_metrics()
            if time.time() - last_adjust >= self.cfg.adjustment_interval:
                await self.make_adjustments()
                last_adjust = time.time()
            await asyncio.sleep(self.cfg.metric_pulling_interval)


def spawn_local_planner(namespace: str, cp_addr: str, cfg: dict) -> subprocess.Popen:
    pc = cfg.get("Planner", {})
    args = [sys.executable, "-m", "dynamo_exp_amd.planner.planner", "--namespace", namespace, "--control-plane",
            cp_addr]
    for k, v in pc.items():
        if k in ("ServiceArgs", "environment"):
            continue
        k = k.replace("_", "-")
        args += [f"--{k}", str(v)] if not isinstance(v, bool) else ([f"--{k}"] if v else [])
    return subprocess.Popen(args, start_new_session=True)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="planner")
    ap.add_argument("--namespace", default="dynamo")
    ap.add_argument("--control-plane", default=None)
    for f, d in PlannerConfig.__dataclass_fields__.items():
        if f in ("namespace",):
            continue
        flag = "--" + f.replace("_", "-")
        if d.type in ("bool",) or isinstance(d.default, bool):
            ap.add_argument(flag, action="store_true")
        else:
            ap.add_argument(flag, type=type(d.default) if d.default is not None else str, default=d.default)
    a, _ = ap.parse_known_args(argv)
    configure_logging()
    cfg = PlannerConfig(**{k: v for k, v in vars(a).items() if k in PlannerConfig.__dataclass_fields__})

    async def run():
        drt = await DistributedRuntime.create(a.control_plane, is_static=True)
        p = await Planner(drt, cfg).start()
        await p.run()

    asyncio.run(run())


if __name__ == "__main__":
    main()
