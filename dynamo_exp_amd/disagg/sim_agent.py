"""KV transfer stand-in for simulated engines (engine/sim.py): the same
control-plane protocol as disagg/agent.py -- the prefill leader publishes
`done{rid, tok, lp}` on `kv_transfer.{ns}.{decode engine}`, the decode
leader turns it into `finish_remote_prefill` -- but no bytes move: the
notification is delayed by the time the layer-streamed RCCL WRITE would
still take after the prefill finished (the last layer group of a request's
KV at the link rate; earlier groups overlap the forward pass).  Used by the
planner benchmark on CPU (tools/planner_bench.py), where the serving graph,
router, queue, planner and supervisor are real and only the GPUs are not.
"""
from __future__ import annotations

import collections
import heapq
import json
import time

import msgpack

from .agent import META_PREFIX

# Llama-3-8B KV bytes per token: 32 layers x K,V x 8 heads x 128 x bf16
BYTES_PER_TOKEN_8B = 32 * 2 * 8 * 128 * 2


class SimKVAgent:
    def __init__(self, engine, cp, engine_id: str, namespace: str = "dynamo", link_GBps: float = 50.0,
                 bytes_per_token: int = BYTES_PER_TOKEN_8B, exposed_fraction: float = 0.25):
        self.engine, self.cp, self.engine_id, self.ns = engine, cp, engine_id, namespace
        self.rank, self.tp = 0, 1
        self.link = link_GBps * 1e9
        self.bytes_per_token = bytes_per_token
        self.exposed = exposed_fraction
        self.inbox: collections.deque = collections.deque()
        self._due: list = []  # (time, seq, dst, msg) notifications still "on the wire"
        self._seq = 0
        self.stats = dict(sent=0, recv=0, reads=0, served=0, deferred=0, sent_bytes=0)
        self.tp_cache: dict[str, int] = {}

    async def start_async(self, cp_async, lease_id: int | None = None) -> "SimKVAgent":
        meta = json.dumps({"engine_id": self.engine_id, "rank": 0, "tp": 1, "backend": "sim"}).encode()
        await cp_async.put(f"{self.ns}/{META_PREFIX}{self.engine_id}/0", meta, lease=lease_id)
        sub = await cp_async.subscribe(f"kv_transfer.{self.ns}.{self.engine_id}")
        import asyncio

        async def pump():
            async for item in sub:
                self.inbox.append(msgpack.unpackb(item["data"], raw=False))

        self._task = asyncio.create_task(pump())
        return self

    # prefill side
    def is_cancelled(self, rid: str) -> bool:
        return False  # the sim decode side never falls back

    def admit(self, rid: str, nblocks: int, read_blocks: int, dst_engine: str) -> bool:
        return True

    def remote_meta(self, r, read_blocks: int) -> dict:
        return {"dst": r.engine_id, "dst_tp": r.engine_tp or None, "skip": r.skip_blocks, "read_blocks": read_blocks}

    def pending_sends(self) -> int:
        return len(self._due)

    def on_prefilled(self, req) -> None:
        nbytes = len(req.prompt) * self.bytes_per_token
        due = time.perf_counter() + self.exposed * nbytes / self.link + 0.0005
        self._seq += 1
        heapq.heappush(self._due, (due, self._seq, req.remote_meta["dst"],
                                   {"t": "done", "rid": req.request_id, "tok": req.output[0], "lp": 0.0}))
        self.stats["sent"] += 1
        self.stats["sent_bytes"] += nbytes

    def flush(self) -> None:
        now = time.perf_counter()
        while self._due and self._due[0][0] <= now:
            _, _, dst, msg = heapq.heappop(self._due)
            self.cp.fire("publish", f"kv_transfer.{self.ns}.{dst}", msgpack.packb(msg))

    # decode side
    def deliver(self) -> None:
        while self.inbox:
            m = self.inbox.popleft()
            if m.get("t") == "done":
                self.engine.finish_remote_prefill(m["rid"], m["tok"], m["lp"])
                self.stats["recv"] += 1

    def pending(self) -> int:
        return len(self._due) + len(self.inbox)


def install_sim_prefill(rep, agent: SimKVAgent):
    rep.engine.prefill_done_hook = agent.on_prefilled
    return agent.flush  # leader step hook (runs while idle too)


def install_sim_decode(rep, agent: SimKVAgent):
    return agent.deliver
