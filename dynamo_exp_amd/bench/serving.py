"""Load generation and timed-window accounting for the serving benchmarks.

Methodology follows the reference's genai-perf runs
(examples/llm/benchmarks/perf.sh:17-54): synthetic ISL/OSL requests with
ignore_eos and min_tokens = max_tokens = OSL, either closed loop at a fixed
concurrency (the sweep) or open loop at a fixed request rate ("p50 TTFT at
fixed QPS", BASELINE.json).  Per request: TTFT = first token - arrival; ITL =
mean gap between consecutive output tokens after the first, i.e.
(t_last - t_first) / (n - 1); percentiles are taken over requests.  Output
throughput = output tokens produced inside the timed window / its length.

Steady state.  A closed loop that starts all streams together runs in lock
step: every stream prefills, decodes and finishes at once, and a short timed
window measures either a prefill storm or a decode-only stretch.  The initial
streams therefore get staggered output lengths (i * OSL / C), so completions
-- and the full ISL/OSL requests that replace them -- are spread uniformly over
an OSL cycle, and the fill phase runs until every staggered stream has been
replaced.  The timed window is counted in engine iterations (one bench "step"
= `iters_per_step` iterations, see bench.py), long enough to average over the
prefill-batching cycle.
"""
from __future__ import annotations

import math
import random
import time
from typing import Callable

import numpy as np


def stagger_lengths(n: int, osl: int) -> list[int]:
    """Output lengths of the initial streams: (i + 1) * osl / n for i < n (the
    last one is a full-length request), i.e. progress spread uniformly."""
    return [max(1, (i + 1) * osl // n) for i in range(n)]


def pct(xs: list[float], p: float) -> float | None:
    if not xs:
        return None
    s = sorted(xs)
    return s[min(len(s) - 1, int(round(p / 100.0 * (len(s) - 1))))]


class PromptGen:
    """Distinct random-token prompts (no accidental prefix sharing), numpy-fast
    so the load generator stays off the engine's critical path."""

    def __init__(self, seed: int, n: int, vocab: int):
        self.rs = np.random.RandomState(seed)
        self.n, self.vocab = n, vocab

    def __call__(self) -> list[int]:
        lo = min(1000, self.vocab // 4)
        return self.rs.randint(lo, self.vocab - lo, size=self.n).tolist()


class _Track:
    __slots__ = ("arrival", "first", "last", "n")

    def __init__(self, arrival: float):
        self.arrival = arrival
        self.first = self.last = None
        self.n = 0


class ServingWindow:
    """Counts tokens and per-request latencies while `counting` is set."""

    def __init__(self, ttft_by_arrival: bool = False):
        # ttft_by_arrival: count a request's TTFT only when it ARRIVED inside
        # the window (open-loop "TTFT at fixed QPS"); default: every first
        # token delivered inside the window (closed loop)
        self.by_arrival = ttft_by_arrival
        self.counting = False
        self.t_start = self.t_end = None
        self.gen = 0
        self.ttft: list[float] = []
        self.req_itl: list[float] = []  # genai-perf ITL: per-request mean gap
        self.step_gap: list[float] = []  # every delivery gap (per-step ITL)
        self.completed = 0

    def open(self) -> None:
        self.t_start = time.perf_counter()
        self.counting = True

    def close(self) -> None:
        self.t_end = time.perf_counter()
        self.counting = False

    @property
    def elapsed(self) -> float:
        if self.t_start is None:
            return 0.0
        return (self.t_end if self.t_end is not None else time.perf_counter()) - self.t_start

    def observe(self, tr: _Track, req, toks, fin: bool) -> None:
        now = time.perf_counter()
        if toks:
            if tr.first is None:
                tr.first = req.first_token_time if req.first_token_time is not None else now
                if self.counting and not (self.by_arrival and tr.arrival < self.t_start):
                    self.ttft.append(tr.first - tr.arrival)
            elif self.counting and tr.last is not None:
                self.step_gap.append((now - tr.last) / len(toks))
            tr.last = now
            tr.n += len(toks)
            if self.counting:
                self.gen += len(toks)
        if fin and self.counting and tr.first is not None and tr.first >= self.t_start:
            self.completed += 1
            if tr.n > 1:
                self.req_itl.append((tr.last - tr.first) / (tr.n - 1))

    def summary(self) -> dict:
        ms = lambda v: None if v is None else round(v * 1000.0, 2)  # noqa: E731
        return {"ttft_p50_ms": ms(pct(self.ttft, 50)), "ttft_p99_ms": ms(pct(self.ttft, 99)),
                "itl_p50_ms": ms(pct(self.req_itl, 50)), "itl_p99_ms": ms(pct(self.req_itl, 99)),
                "step_itl_p50_ms": ms(pct(self.step_gap, 50)),
                "itl_mean_ms": ms(sum(self.step_gap) / len(self.step_gap) if self.step_gap else None),
                "completed_requests": self.completed}

    def state(self) -> dict:
        """Raw samples for the cross-rank merge (disaggregated bench)."""
        return {"gen": self.gen, "elapsed": self.elapsed, "ttft": self.ttft, "req_itl": self.req_itl,
                "step_gap": self.step_gap, "completed": self.completed}

    @classmethod
    def merged(cls, states: list[dict]) -> "ServingWindow":
        """All ranks' samples; the window is the longest rank window."""
        w = cls()
        w.t_start, w.t_end = 0.0, max([s["elapsed"] for s in states] or [0.0])
        for s in states:
            w.gen += s["gen"]
            w.ttft += s["ttft"]
            w.req_itl += s["req_itl"]
            w.step_gap += s["step_gap"]
            w.completed += s["completed"]
        return w


class LoadGen:
    """Feeds an engine with ISL/OSL requests.

    add(rid, prompt, params, on_output) submits one request to the engine.
    Closed loop (`start_closed(C)`): C streams, each replaced by a new request
    when it finishes.  Open loop (`start_open(qps)`): Poisson arrivals at
    `qps` requests/s, submitted by `poll()` (call it before every engine
    step); `next_arrival_in()` tells an idle driver how long to sleep."""

    def __init__(self, add: Callable, gen_prompt: Callable[[], list[int]], osl: int, window: ServingWindow,
                 rid_prefix: str = "r", seed: int = 0):
        self.add = add
        self.gen_prompt = gen_prompt
        self.osl = osl
        self.win = window
        self.prefix = rid_prefix
        self.n = 0
        self.fill = 0  # staggered initial streams still running
        self.admitting = True
        self.qps = None
        self._next = math.inf
        self._rng = random.Random(seed)

    def _params(self, osl: int):
        from ..engine.request import SamplingParams

        return SamplingParams(temperature=0.0, max_tokens=osl, min_tokens=osl, ignore_eos=True)

    def submit(self, osl: int | None = None, arrival: float | None = None) -> None:
        if not self.admitting:
            return
        self.n += 1
        rid = f"{self.prefix}{self.n}"
        osl = osl or self.osl
        tr = _Track(arrival if arrival is not None else time.perf_counter())
        closed = self.qps is None
        staggered = osl != self.osl

        def on_output(req, toks, lps, fin):
            self.win.observe(tr, req, toks, fin)
            if fin:
                if staggered:
                    self.fill -= 1
                if closed:
                    self.submit()

        self.add(rid, self.gen_prompt(), self._params(osl), on_output)

    # closed loop
    def start_closed(self, concurrency: int) -> None:
        lens = stagger_lengths(concurrency, self.osl)
        self.fill = sum(1 for o in lens if o != self.osl)
        for o in lens:
            self.submit(o)

    @property
    def filling(self) -> bool:
        return self.fill > 0

    # open loop
    def start_open(self, qps: float) -> None:
        self.qps = float(qps)
        self._next = time.perf_counter() + self._rng.expovariate(self.qps)

    def poll(self) -> int:
        """Submit every arrival that is due; returns how many."""
        if self.qps is None or not self.admitting:
            return 0
        now = time.perf_counter()
        k = 0
        while self._next <= now:
            self.submit(arrival=self._next)
            self._next += self._rng.expovariate(self.qps)
            k += 1
        return k

    def next_arrival_in(self) -> float:
        return max(0.0, self._next - time.perf_counter()) if self.qps is not None else 0.0

    def stop(self) -> None:
        self.admitting = False


def drive(eng, load, win, args, sync, barrier=lambda: None, service=lambda: None, tag="", log=lambda m: None):
    """Fill to steady state, W warmup steps, K timed steps.  `service()` runs
    before every engine iteration (disagg: KV receive bookkeeping).  Returns
    the engine stats delta over the window."""
    ips = max(1, args.iters_per_step)
    beat = {"t": time.perf_counter(), "phase": "fill"}

    def iterate(n):
        done = 0
        while done < n:
            now = time.perf_counter()
            if now - beat["t"] > 20.0:  # progress line for long phases (slow rehearsals, big fills)
                beat["t"] = now
                log(f"{tag}{beat['phase']}: {eng.stats['steps']} engine iterations, {win.gen} tokens")
            load.poll()
            service()
            if eng.has_pending_work():
                n0 = eng.stats["steps"]
                eng.step()
                done += eng.stats["steps"] > n0  # iterations that ran a batch
            else:
                time.sleep(min(0.002, max(0.0001, load.next_arrival_in())))

    t0 = time.perf_counter()
    if load.qps is None:
        n = 0
        while load.filling:
            iterate(1)
            n += 1
    else:  # open loop: populate the pipeline (about one OSL of decode iterations)
        n = 2 * args.osl
        iterate(n)
    log(f"{tag}steady-state fill: {n} iterations in {time.perf_counter() - t0:.1f}s")
    beat["phase"] = "warmup"
    iterate(args.warmup * ips)
    sync()
    barrier()
    s0 = dict(eng.stats)
    win.open()
    beat["phase"] = "timed window"
    per_step = []
    for _ in range(args.steps):
        g0, ts = win.gen, time.perf_counter()
        iterate(ips)
        if args.trace_steps:
            sync()
            per_step.append(round((win.gen - g0) / (time.perf_counter() - ts), 1))
    sync()
    win.close()
    if per_step:
        log(f"{tag}per-step tok/s: {per_step}")
    s1 = eng.stats
    return {k: s1.get(k, 0) - s0.get(k, 0)
            for k in ("prefill_steps", "decode_steps", "mixed_steps", "steps", "prefill_step_tokens")}


def fixed_qps_segment(eng, add, gen_prompt, osl: int, qps: float, seconds: float, warm: float = 3.0,
                      service=lambda: None, sync=lambda: None, rid_prefix: str = "q", seed: int = 0,
                      log=lambda m: None) -> ServingWindow:
    """Open-loop Poisson arrivals at `qps` requests/s (the reference's "p50
    TTFT at fixed QPS", BASELINE.json metric): `warm` seconds to populate the
    engine, then `seconds` measured.  TTFT counts requests that arrived inside
    the measured span and got their first token before it closed; the
    caller starts from an engine whose earlier load was stopped."""
    win = ServingWindow(ttft_by_arrival=True)
    load = LoadGen(add, gen_prompt, osl, win, rid_prefix=rid_prefix, seed=seed)
    load.start_open(qps)
    t0 = time.perf_counter()
    opened = False
    while True:
        now = time.perf_counter()
        if not opened and now - t0 >= warm:
            sync()
            win.open()
            opened = True
        if opened and now - t0 >= warm + seconds:
            break
        load.poll()
        service()
        if eng.has_pending_work():
            eng.step()
        else:
            time.sleep(min(0.002, max(0.0001, load.next_arrival_in())))
    sync()
    win.close()
    load.stop()
    log(f"fixed-QPS segment: {qps:.2f} req/s, {load.n} arrivals, TTFT p50 "
        f"{win.summary()['ttft_p50_ms']} ms over {len(win.ttft)} requests")
    return win


def closed_loop_request_rate(win: ServingWindow, osl: int) -> float:
    """Requests/s the closed loop sustained: output tokens / OSL / window."""
    return win.gen / max(1, osl) / win.elapsed if win.elapsed > 0 else 0.0
