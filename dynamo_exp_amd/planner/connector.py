"""Planner connectors (reference components/planner/src/dynamo/planner/
{planner_connector.py, local_connector.py}).

`LocalConnector` talks to the `serve` supervisor of the namespace over the
control plane (subject `supervisor.{ns}`):
  add_component(Svc)    -> new watcher `{ns}_{Svc}_{n}` on a free GPU;
  remove_component(Svc) -> revoke the newest worker's lease (its endpoints
                           vanish from routers; a decode worker drains its
                           in-flight streams, a prefill worker stops pulling the
                           queue and finishes its current work), wait for it to
                           exit, then remove the watcher.
"""
from __future__ import annotations

import abc
import asyncio
import json
import logging
import os
import time
import uuid

from ..sdk.state import read_state

log = logging.getLogger("dynamo_exp_amd.planner")


class PlannerConnector(abc.ABC):
    @abc.abstractmethod
    async def add_component(self, component_name: str) -> bool: ...

    @abc.abstractmethod
    async def remove_component(self, component_name: str) -> bool: ...


class LocalConnector(PlannerConnector):
    def __init__(self, namespace: str, drt, gpus_per_worker: float | None = None, timeout: float = 120.0):
        """gpus_per_worker None: the supervisor gives an added worker its service's configured GPU share."""
        self.ns = namespace
        self.drt = drt
        self.gpus = gpus_per_worker
        self.timeout = timeout

    async def _cmd(self, **cmd) -> dict:
        reply = f"supervisor/replies/{uuid.uuid4().hex}"
        cmd["reply"] = reply
        await self.drt.cp.publish(f"supervisor.{self.ns}", json.dumps(cmd).encode())
        end = time.time() + self.timeout
        while time.time() < end:
            raw = await self.drt.cp.get(reply)
            if raw is not None:
                await self.drt.cp.delete(reply)
                return json.loads(raw)
            await asyncio.sleep(0.1)
        return {"ok": False, "error": "supervisor timeout"}

    def _watchers(self, component: str) -> list[str]:
        st = read_state(self.ns)
        return sorted(n for n, w in (st.get("watchers") or {}).items() if w["service"] == component)

    async def add_component(self, component_name: str) -> bool:
        existing = self._watchers(component_name)
        n = 0
        while f"{self.ns}_{component_name}_{n}" in existing:
            n += 1
        extra = {} if self.gpus is None else {"gpus": self.gpus}
        res = await self._cmd(op="add", name=f"{self.ns}_{component_name}_{n}", service=component_name,
                              numprocesses=1, **extra)
        if not res.get("ok"):
            log.warning("add %s failed: %s", component_name, res.get("error"))
        return bool(res.get("ok"))

    async def remove_component(self, component_name: str, drain_timeout: float = 120.0) -> bool:
        """Graceful scale-down (reference local_connector.py:197-325): the
        supervisor stops respawning the watcher, the worker's lease is revoked
        -- its endpoints vanish from every router, a decode worker finishes its
        in-flight streams, a prefill worker stops pulling the queue and
        finishes what it dequeued -- the worker exits by itself, then the
        watcher is removed (anything still alive after `drain_timeout` is
        terminated)."""
        names = self._watchers(component_name)
        if not names:
            return False
        name = names[-1]
        st = read_state(self.ns)
        pids = st["watchers"][name]["pids"]
        leases = [w["lease"] for w in (st.get("components", {}).get(component_name, {}).get("workers", {}).values())
                  if w.get("pid") in pids]
        await self._cmd(op="retire", name=name)
        for lid in leases:  # graceful: the worker drains when its lease dies
            try:
                await self.drt.cp.lease_revoke(lid)
            except Exception:
                pass
        end = time.time() + drain_timeout
        while time.time() < end and any(_alive(p) for p in pids):
            await asyncio.sleep(0.5)
        res = await self._cmd(op="remove", name=name, timeout=30)
        return bool(res.get("ok"))


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] not in ("Z", "X")
    except OSError:
        return False
