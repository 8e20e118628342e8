"""Tracing and per-request timing (SURVEY §5.1 build target; the reference has
no tracing beyond logs, `lib/llm/src/http/service/openai.rs:243`).

* roctx ranges: `span("engine.step/mixed")` pushes/pops a ROCTx range so the
  engine step, sampling and P->D KV transfers show up on the timeline of
  `rocprofv3 --kernel-trace --marker-trace`.  Enabled with DX_ROCTX=1 (the
  ctypes call costs ~1 us, so it is off by default); libroctx64 is loaded
  lazily and a missing library just disables the ranges.
* `RequestTimer`: Prometheus histograms of per-request phases -- queue
  (arrival -> admitted), prefill (admitted -> first token), decode (first ->
  last token), end-to-end, KV transfer time / bytes -- on a registry the
  worker's metrics endpoint exposes.
* `stage(name, request_id)`: per-request stage timestamps across processes
  (HTTP receive, request-plane send / receive / first frame, engine arrival /
  admit / first token), appended to `$DX_STAGE_TRACE.<pid>.jsonl` when that
  variable is set -- CLOCK_MONOTONIC, so the files of all the processes of
  one host join on the request id (tools/stage_report.py).
"""
from __future__ import annotations

import atexit
import contextlib
import ctypes
import json
import os
import threading
import time

from prometheus_client import CollectorRegistry, Counter, Histogram

_lib = None
_lock = threading.Lock()


def _roctx():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                lib = False
                if os.environ.get("DX_ROCTX", "0") not in ("", "0"):
                    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
                        try:
                            lib = ctypes.CDLL(name)
                            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                            break
                        except OSError:
                            lib = False
                _lib = lib
    return _lib or None


def enabled() -> bool:
    return _roctx() is not None


def range_push(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def range_pop() -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePop()


def mark(msg: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(msg.encode())


@contextlib.contextmanager
def span(name: str):
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


_STAGE_PATH = os.environ.get("DX_STAGE_TRACE") or None
_stages: list = []


def stage(name: str, request_id, t: float | None = None) -> None:
    if _STAGE_PATH is None or request_id is None:
        return
    _stages.append((name, request_id, time.perf_counter() if t is None else t))
    if len(_stages) >= 2048:
        flush_stages()


def flush_stages() -> None:
    global _stages
    if not _stages:
        return
    rows, _stages = _stages, []
    with open(f"{_STAGE_PATH}.{os.getpid()}.jsonl", "a") as f:
        f.write("".join(json.dumps(r) + "\n" for r in rows))


if _STAGE_PATH is not None:
    atexit.register(flush_stages)


_LAT_BUCKETS = (.001, .0025, .005, .01, .025, .05, .1, .25, .5, 1, 2.5, 5, 10, 30, 60, 120)


class RequestTimer:
    """Histograms of request phases; `observe(req)` when a request finishes."""

    def __init__(self, registry: CollectorRegistry | None = None, prefix: str = "dynamo_engine"):
        self.registry = r = registry or CollectorRegistry()
        self.queue = Histogram(f"{prefix}_queue_seconds", "arrival -> admitted", buckets=_LAT_BUCKETS, registry=r)
        self.prefill = Histogram(f"{prefix}_prefill_seconds", "admitted -> first token", buckets=_LAT_BUCKETS,
                                 registry=r)
        self.ttft = Histogram(f"{prefix}_time_to_first_token_seconds", "arrival -> first token",
                              buckets=_LAT_BUCKETS, registry=r)
        self.decode = Histogram(f"{prefix}_decode_seconds", "first -> last token", buckets=_LAT_BUCKETS, registry=r)
        self.e2e = Histogram(f"{prefix}_request_seconds", "arrival -> finish", buckets=_LAT_BUCKETS, registry=r)
        self.itl = Histogram(f"{prefix}_inter_token_seconds", "mean inter-token latency per request",
                             buckets=_LAT_BUCKETS, registry=r)
        self.kv_xfer = Histogram(f"{prefix}_kv_transfer_seconds", "P->D KV transfer time", buckets=_LAT_BUCKETS,
                                 registry=r)
        self.kv_bytes = Counter(f"{prefix}_kv_transfer_bytes", "P->D KV bytes moved", registry=r)
        self.finished = Counter(f"{prefix}_requests_finished", "finished requests", ["reason"], registry=r)

    def observe(self, req) -> None:
        a = req.arrival
        adm = getattr(req, "admit_time", None)
        ft, fin = req.first_token_time, req.finish_time or time.perf_counter()
        if _STAGE_PATH is not None:
            rid = getattr(req, "request_id", None)
            stage("eng.arrival", rid, a)
            if adm is not None:
                stage("eng.admit", rid, adm)
            if ft is not None:
                stage("eng.first", rid, ft)
            stage("eng.finish", rid, fin)
        if adm is not None:
            self.queue.observe(max(0.0, adm - a))
            if ft is not None:
                self.prefill.observe(max(0.0, ft - adm))
        if ft is not None:
            self.ttft.observe(max(0.0, ft - a))
            self.decode.observe(max(0.0, fin - ft))
            n = len(req.output)
            if n > 1:
                self.itl.observe(max(0.0, fin - ft) / (n - 1))
        self.e2e.observe(max(0.0, fin - a))
        self.finished.labels(str(getattr(req.finish_reason, "value", req.finish_reason))).inc()

    def observe_transfer(self, seconds: float, nbytes: int) -> None:
        self.kv_xfer.observe(seconds)
        self.kv_bytes.inc(nbytes)
