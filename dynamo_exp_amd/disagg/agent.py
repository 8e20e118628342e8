"""Serving-time KV transfer between independently started worker processes
(the reference's NIXL connector + NixlMetadataStore).

Each worker's agent hosts a c10d TCPStore and publishes its metadata under
`{ns}/kv_transfer/{engine_id}` (lease-bound).  A prefill->decode pair gets its
own 2-rank process group built directly on a PrefixStore of the decode
worker's store (rank 0 = prefill, rank 1 = decode): ProcessGroupNCCL (RCCL
over xGMI) on GPUs, ProcessGroupGloo over host staging on CPU.  Pairs are
created lazily at the first transfer, so workers may join and leave freely
(no global communicator rebuild -- SURVEY §7.4 item 4).

Protocol per request (same as the bench path, see transfer.py):
  P: pack blocks -> publish notify{rid, src, nbytes, tok, lp} on
     `kv_transfer.{dst}` -> pg.send                     (engine thread)
  D: notify -> pg.recv into staging -> on completion unpack into the
     pre-allocated blocks -> engine.finish_remote_prefill (engine thread hook)
"""
from __future__ import annotations

import asyncio
import collections
import datetime
import json
import logging
import socket
import time

import msgpack
import torch
import torch.distributed as dist

from ..utils import tracing
from ..utils.faults import FAULTS
from .transfer import pack_blocks, transfer_bytes, unpack_blocks

log = logging.getLogger("dynamo_exp_amd.disagg.agent")

META_PREFIX = "kv_transfer/"


class _Pair:
    def __init__(self, pg, rank: int):
        self.pg, self.rank = pg, rank


class KVTransferAgent:
    def __init__(self, engine, cp, loop: asyncio.AbstractEventLoop, engine_id: str, namespace: str = "dynamo",
                 host: str | None = None):
        self.engine = engine
        self.cp = cp
        self.loop = loop
        self.engine_id = engine_id
        self.ns = namespace
        self.kv = engine.runner.kv_cache
        self.gpu = self.kv.is_cuda
        import os

        self.host = host or os.environ.get("DX_HOST_IP", "127.0.0.1")
        self.store = dist.TCPStore(self.host, 0, is_master=True, wait_for_workers=False,
                                   timeout=datetime.timedelta(seconds=120))
        self.pairs: dict[str, _Pair] = {}
        self.meta_cache: dict[str, dict] = {}
        self.inbox: collections.deque = collections.deque()
        self.sends: collections.deque = collections.deque()
        self.recvs: collections.deque = collections.deque()
        self.stats = dict(sent=0, recv=0, sent_bytes=0, recv_bytes=0)
        self._sub_task = None

    # --------------------------------------------------------------- metadata
    @property
    def meta_key(self) -> str:
        return f"{self.ns}/{META_PREFIX}{self.engine_id}"

    async def start(self, lease_id: int | None = None) -> "KVTransferAgent":
        meta = {"engine_id": self.engine_id, "host": self.host, "port": self.store.port,
                "backend": "nccl" if self.gpu else "gloo"}
        await self.cp.put(self.meta_key, json.dumps(meta).encode(), lease=lease_id)
        sub = await self.cp.subscribe(f"kv_transfer.{self.ns}.{self.engine_id}")

        async def pump():
            async for item in sub:
                self.inbox.append(msgpack.unpackb(item["data"], raw=False))

        self._sub_task = asyncio.create_task(pump())
        return self

    def _meta(self, engine_id: str) -> dict:
        m = self.meta_cache.get(engine_id)
        if m is None:
            fut = asyncio.run_coroutine_threadsafe(self.cp.get(f"{self.ns}/{META_PREFIX}{engine_id}"), self.loop)
            raw = fut.result(30)
            if raw is None:
                raise RuntimeError(f"no kv_transfer metadata for engine {engine_id}")
            m = json.loads(raw)
            self.meta_cache[engine_id] = m
        return m

    def _pair(self, peer: str, role: str) -> _Pair:
        """role 'prefill': I am rank 0 and connect to the peer's (decode) store."""
        key = f"{role}:{peer}"
        p = self.pairs.get(key)
        if p is not None:
            return p
        if role == "prefill":
            m = self._meta(peer)
            store = dist.TCPStore(m["host"], m["port"], is_master=False, timeout=datetime.timedelta(seconds=120))
            prefix = f"pair/{self.engine_id}/{peer}"
            rank = 0
        else:
            store = self.store
            prefix = f"pair/{peer}/{self.engine_id}"
            rank = 1
        ps = dist.PrefixStore(prefix, store)
        timeout = datetime.timedelta(seconds=300)
        pg = dist.ProcessGroupNCCL(ps, rank, 2, timeout) if self.gpu else dist.ProcessGroupGloo(ps, rank, 2, timeout)
        p = _Pair(pg, rank)
        self.pairs[key] = p
        return p

    # --------------------------------------------------------------- prefill side
    def send(self, rid: str, block_ids: list[int], dst_engine: str, first_token: int, logprob: float) -> None:
        """Engine thread: ship KV of `block_ids` to the decode engine."""
        FAULTS.before_kv_transfer_sync()
        nbytes = transfer_bytes(self.kv, len(block_ids))
        note = msgpack.packb({"rid": rid, "src": self.engine_id, "nbytes": nbytes, "tok": first_token, "lp": logprob})
        asyncio.run_coroutine_threadsafe(self.cp.publish(f"kv_transfer.{self.ns}.{dst_engine}", note), self.loop)
        pair = self._pair(dst_engine, "prefill")
        with tracing.span("kv_transfer.send"):
            buf = pack_blocks(self.kv, block_ids)
            if not self.gpu:
                buf = buf.cpu()
            work = pair.pg.send([buf], 1, 0)
        self.sends.append((rid, work, buf))
        self.stats["sent"] += 1
        self.stats["sent_bytes"] += nbytes

    def poll_sends(self) -> list[str]:
        done = []
        while self.sends and self._done(self.sends[0][1]):
            rid, _, _ = self.sends.popleft()
            done.append(rid)
        return done

    # --------------------------------------------------------------- decode side
    def service(self) -> None:
        """Engine-thread hook: post receives for notifications, finish landed ones."""
        eng = self.engine
        while self.inbox:
            m = self.inbox.popleft()
            req = eng.scheduler.remote.get(m["rid"])
            if req is None:  # request was cancelled; still drain the bytes
                blocks = None
            else:
                bs = eng.kv.block_size
                skip = req.num_computed // bs
                blocks = req.block_ids[skip:(len(req.prompt) + bs - 1) // bs]
            pair = self._pair(m["src"], "decode")
            buf = torch.empty(m["nbytes"], dtype=torch.uint8, device=self.kv.device if self.gpu else "cpu")
            work = pair.pg.recv([buf], 0, 0)
            m["t0"] = time.perf_counter()
            self.recvs.append((m, work, buf, blocks))
        while self.recvs and self._done(self.recvs[0][1]):
            m, work, buf, blocks = self.recvs.popleft()
            if self.gpu:
                work.wait()
            if blocks is not None:
                with tracing.span("kv_transfer.unpack"):
                    unpack_blocks(self.kv, buf if self.gpu else buf.to(self.kv.device), blocks)
                eng.finish_remote_prefill(m["rid"], m["tok"], m["lp"])
            eng.request_timer.observe_transfer(time.perf_counter() - m["t0"], m["nbytes"])
            self.stats["recv"] += 1
            self.stats["recv_bytes"] += m["nbytes"]

    def _done(self, work) -> bool:
        if not self.gpu:
            work.wait()
            return True
        return work.is_completed()

    def pending(self) -> int:
        return len(self.sends) + len(self.recvs) + len(self.inbox)
