"""Fault injection for resilience tests (SURVEY §5.3 build target; the
reference has none).

Faults are armed programmatically (`FAULTS.arm("kv_transfer.delay_ms", 200)`)
or from the environment of a worker process:

    DX_FAULTS="worker.exit_after_requests=3,kv_transfer.delay_ms=200,endpoint.error_rate=0.1,lease.drop_after_s=5"

Hook points (each a no-op unless armed):
  worker.exit_after_requests  N   hard-exit (code 137) when the N-th request starts -- a crashed worker
  lease.drop_after_s          S   revoke the primary lease S seconds after start -- a partitioned worker
  endpoint.error_rate         P   raise InjectedFault in a request handler with probability P
  kv_transfer.delay_ms        MS  sleep before every P->D KV send
  kv_transfer.fail_rate       P   fail a P->D KV send with probability P
  engine.step_delay_ms        MS  stall each engine step (slow GPU / straggler)
  kv_transfer.corrupt_pieces  N   flip one byte of each of the next N received KV pieces before
                                  they are unpacked (a mis-placed / damaged transfer: the bench
                                  preflight and --verify-tokens must catch it)
"""
from __future__ import annotations

import asyncio
import logging
import os
import random
import threading
import time

log = logging.getLogger("dynamo_exp_amd.faults")


class InjectedFault(RuntimeError):
    pass


class FaultInjector:
    def __init__(self, spec: str | None = None, seed: int | None = None):
        self.armed: dict[str, float] = {}
        self.counts: dict[str, int] = {}
        self.rng = random.Random(seed)
        self._lock = threading.Lock()
        if spec:
            for item in spec.split(","):
                if "=" in item:
                    k, v = item.split("=", 1)
                    self.arm(k.strip(), float(v))

    def arm(self, name: str, value: float = 1.0) -> None:
        self.armed[name] = float(value)
        log.warning("fault armed: %s=%s", name, value)

    def disarm(self, name: str | None = None) -> None:
        if name is None:
            self.armed.clear()
        else:
            self.armed.pop(name, None)

    def value(self, name: str) -> float | None:
        return self.armed.get(name)

    def _tick(self, name: str) -> int:
        with self._lock:
            self.counts[name] = self.counts.get(name, 0) + 1
            return self.counts[name]

    # ---------------------------------------------------------------- hooks
    def on_request(self) -> None:
        n = self._tick("requests")
        lim = self.armed.get("worker.exit_after_requests")
        if lim is not None and n >= lim:
            log.error("fault: worker exit after %d requests", n)
            os._exit(137)
        p = self.armed.get("endpoint.error_rate")
        if p and self.rng.random() < p:
            raise InjectedFault("injected endpoint error")

    async def before_kv_transfer(self) -> None:
        d = self.armed.get("kv_transfer.delay_ms")
        if d:
            await asyncio.sleep(d / 1000.0)
        p = self.armed.get("kv_transfer.fail_rate")
        if p and self.rng.random() < p:
            raise InjectedFault("injected kv transfer failure")

    def before_kv_transfer_sync(self) -> None:
        d = self.armed.get("kv_transfer.delay_ms")
        if d:
            time.sleep(d / 1000.0)
        p = self.armed.get("kv_transfer.fail_rate")
        if p and self.rng.random() < p:
            raise InjectedFault("injected kv transfer failure")

    def corrupt_received(self, buf) -> None:
        """Data plane, before unpacking a received buffer: damage it while
        `kv_transfer.corrupt_pieces` has pieces left (a device op, no sync)."""
        n = self.armed.get("kv_transfer.corrupt_pieces")
        if not n or buf is None or buf.numel() == 0:
            return
        with self._lock:
            self.armed["kv_transfer.corrupt_pieces"] = n - 1
        k = buf.numel() // 2
        buf[k:k + 1].bitwise_not_()
        log.error("fault: corrupted a received KV piece (%d bytes)", buf.numel())

    def on_engine_step(self) -> None:
        d = self.armed.get("engine.step_delay_ms")
        if d:
            time.sleep(d / 1000.0)

    def start_lease_dropper(self, drt) -> asyncio.Task | None:
        s = self.armed.get("lease.drop_after_s")
        if s is None or drt.primary_lease is None:
            return None

        async def drop():
            await asyncio.sleep(s)
            log.error("fault: revoking primary lease %x", drt.primary_lease.id)
            await drt.primary_lease.revoke()

        return asyncio.create_task(drop())


FAULTS = FaultInjector(os.environ.get("DX_FAULTS"))
