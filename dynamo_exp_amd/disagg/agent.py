"""Serving-time KV transfer between independently started workers, per TP rank
(the reference's NIXL connector + NixlMetadataStore + per-rank notification
counting; patch :1296-1424, :2991, :3252-3255).

Every TP rank of a worker owns one `KVTransferAgent`: it hosts a c10d
TCPStore and publishes `{ns}/kv_transfer/{engine_id}/{rank}` (lease-bound)
with its address and the worker's TP size.  A (prefill rank, decode rank)
pair gets its own 2-rank process group built on a PrefixStore of the decode
rank's store -- ProcessGroupNCCL (RCCL over xGMI) on GPUs, ProcessGroupGloo
with host staging on CPU -- created lazily at the first transfer, so workers
join and leave without any global communicator rebuild.

TP layouts: the KV cache block is [Hkv_local][BS][D], so a rank's KV heads are
one contiguous byte range of every block and `tp_relayout_plan` turns a
(prefill TP, decode TP) pair into (src rank, dst rank, src offset, dst offset,
length) pieces.  Prefill rank r packs and sends the pieces it owns; decode rank
d receives the pieces addressed to it and unpacks them at their offset -- the
kv_rearrange relayout of the reference, fused into the pack/unpack kernel.

Protocol per request:
  P (every rank, lockstep): prefill done -> pack pieces -> pg.send; rank 0
     publishes notify{rid, src, src_tp, nblocks, tok, lp} on
     `kv_transfer.{ns}.{dst}`; the blocks are released right after the pack
     (the send reads the staging copy).
  D leader: notify -> ext event "kv_recv" -> every decode rank posts its
     receives (same order on every pair); when the leader's receives landed
     -> ext event "kv_finish" -> every rank orders its compute stream after
     its receive, unpacks into the request's blocks, finish_remote_prefill --
     the same step on every rank, so the TP schedulers never diverge.
"""
from __future__ import annotations

import asyncio
import collections
import datetime
import json
import logging
import os
import time

import msgpack
import torch
import torch.distributed as dist

from ..utils import tracing
from ..utils.faults import FAULTS
from .transfer import pack_blocks, tp_relayout_plan, unpack_blocks

log = logging.getLogger("dynamo_exp_amd.disagg.agent")

META_PREFIX = "kv_transfer/"


class _Pair:
    def __init__(self, pg, rank: int):
        self.pg, self.rank = pg, rank


class _CP:
    """Blocking control-plane calls from a non-event-loop thread."""

    def __init__(self, client, loop: asyncio.AbstractEventLoop):
        self.client, self.loop = client, loop

    def call(self, name: str, *a, **kw):
        return asyncio.run_coroutine_threadsafe(getattr(self.client, name)(*a, **kw), self.loop).result(30)

    def fire(self, name: str, *a, **kw) -> None:
        asyncio.run_coroutine_threadsafe(getattr(self.client, name)(*a, **kw), self.loop)


class KVTransferAgent:
    def __init__(self, engine, cp: _CP, engine_id: str, namespace: str = "dynamo", tp_rank: int = 0,
                 tp_size: int = 1, host: str | None = None):
        self.engine = engine  # this rank's LLMEngine
        self.cp = cp
        self.engine_id = engine_id
        self.ns = namespace
        self.rank, self.tp = tp_rank, tp_size
        self.kv = engine.runner.kv_cache
        self.gpu = self.kv.is_cuda
        mc = engine.model.cfg
        self.total_kv_heads = mc.num_key_value_heads
        self.block_size = self.kv.shape[4]
        self.head_dim = self.kv.shape[5]
        self.host = host or os.environ.get("DX_HOST_IP", "127.0.0.1")
        self.store = dist.TCPStore(self.host, 0, is_master=True, wait_for_workers=False,
                                   timeout=datetime.timedelta(seconds=120))
        self.pairs: dict[tuple, _Pair] = {}
        self.meta_cache: dict[tuple, dict] = {}
        self.plans: dict[tuple, list] = {}
        self.inbox: collections.deque = collections.deque()  # leader: notifications
        self.sends: collections.deque = collections.deque()
        self.recvs: dict[str, dict] = {}  # rid -> {"works": [(work, buf, piece)], "blocks", "m"}
        self.stats = dict(sent=0, recv=0, sent_bytes=0, recv_bytes=0)

    # --------------------------------------------------------------- metadata
    @property
    def meta_key(self) -> str:
        return f"{self.ns}/{META_PREFIX}{self.engine_id}/{self.rank}"

    def meta(self) -> bytes:
        return json.dumps({"engine_id": self.engine_id, "rank": self.rank, "tp": self.tp, "host": self.host,
                           "port": self.store.port, "backend": "nccl" if self.gpu else "gloo"}).encode()

    async def start_async(self, cp_async, lease_id: int | None = None) -> "KVTransferAgent":
        """Leader (rank 0), inside the worker's event loop: publish metadata and
        listen for notifications addressed to this engine."""
        await cp_async.put(self.meta_key, self.meta(), lease=lease_id)
        sub = await cp_async.subscribe(f"kv_transfer.{self.ns}.{self.engine_id}")

        async def pump():
            async for item in sub:
                self.inbox.append(msgpack.unpackb(item["data"], raw=False))

        self._sub_task = asyncio.create_task(pump())
        return self

    def start_sync(self, lease_id: int | None = None) -> "KVTransferAgent":
        """Follower ranks: publish metadata only (notifications reach the leader)."""
        self.cp.call("put", self.meta_key, self.meta(), lease=lease_id)
        return self

    def _meta(self, engine_id: str, rank: int) -> dict:
        key = (engine_id, rank)
        m = self.meta_cache.get(key)
        if m is None:
            t0 = time.time()
            while True:
                raw = self.cp.call("get", f"{self.ns}/{META_PREFIX}{engine_id}/{rank}")
                if raw is not None:
                    break
                if time.time() - t0 > 30:
                    raise RuntimeError(f"no kv_transfer metadata for engine {engine_id} rank {rank}")
                time.sleep(0.05)
            m = self.meta_cache[key] = json.loads(raw)
        return m

    def _plan(self, prefill_tp: int, decode_tp: int) -> list:
        key = (prefill_tp, decode_tp)
        p = self.plans.get(key)
        if p is None:
            p = self.plans[key] = tp_relayout_plan(prefill_tp, decode_tp, self.total_kv_heads, self.block_size,
                                                   self.head_dim, self.kv.element_size())
        return p

    def _pair(self, peer: str, peer_rank: int, role: str) -> _Pair:
        """role 'prefill': I am rank 0 of the pair and connect to the peer's (decode) store."""
        key = (role, peer, peer_rank)
        p = self.pairs.get(key)
        if p is not None:
            return p
        if role == "prefill":
            m = self._meta(peer, peer_rank)
            store = dist.TCPStore(m["host"], m["port"], is_master=False, timeout=datetime.timedelta(seconds=120))
            prefix = f"pair/{self.engine_id}.{self.rank}/{peer}.{peer_rank}"
            rank = 0
        else:
            store = self.store
            prefix = f"pair/{peer}.{peer_rank}/{self.engine_id}.{self.rank}"
            rank = 1
        ps = dist.PrefixStore(prefix, store)
        timeout = datetime.timedelta(seconds=300)
        pg = dist.ProcessGroupNCCL(ps, rank, 2, timeout) if self.gpu else dist.ProcessGroupGloo(ps, rank, 2, timeout)
        p = self.pairs[key] = _Pair(pg, rank)
        return p

    def _piece_bytes(self, piece, nblocks: int) -> int:
        L = self.kv.shape[0]
        return L * 2 * nblocks * piece.nbytes

    # --------------------------------------------------------------- prefill side
    def send(self, rid: str, block_ids: list[int], dst_engine: str, first_token: int, logprob: float) -> None:
        """Engine thread, every prefill rank (lockstep): ship this rank's pieces."""
        FAULTS.before_kv_transfer_sync()
        dst_tp = self._meta(dst_engine, 0)["tp"]
        if self.rank == 0:
            note = msgpack.packb({"rid": rid, "src": self.engine_id, "src_tp": self.tp, "nblocks": len(block_ids),
                                  "tok": first_token, "lp": logprob})
            self.cp.fire("publish", f"kv_transfer.{self.ns}.{dst_engine}", note)
        with tracing.span("kv_transfer.send"):
            for piece in self._plan(self.tp, dst_tp):
                if piece.src_rank != self.rank:
                    continue
                pair = self._pair(dst_engine, piece.dst_rank, "prefill")
                buf = pack_blocks(self.kv, block_ids, inner_off=piece.src_inner_off, inner_bytes=piece.nbytes)
                if not self.gpu:
                    buf = buf.cpu()
                work = pair.pg.send([buf], 1, 0)
                self.sends.append((rid, work, buf))
                self.stats["sent_bytes"] += buf.numel()
        self.stats["sent"] += 1

    def poll_sends(self) -> int:
        """Release staging buffers of completed sends; returns how many are still in flight."""
        while self.sends and self._done(self.sends[0][1]):
            self.sends.popleft()
        return len(self.sends)

    # --------------------------------------------------------------- decode side
    def take_notifications(self) -> list[dict]:
        out = []
        while self.inbox:
            out.append(self.inbox.popleft())
        return out

    def post_recv(self, m: dict) -> None:
        """Every decode rank (lockstep): post the receives of request m['rid']."""
        eng = self.engine
        req = eng.scheduler.remote.get(m["rid"])
        if req is None:  # cancelled meanwhile: still drain the bytes
            blocks = None
        else:
            bs = eng.kv.block_size
            skip = req.num_computed // bs
            blocks = req.block_ids[skip:(len(req.prompt) + bs - 1) // bs]
            assert len(blocks) == m["nblocks"], (len(blocks), m["nblocks"])
        works = []
        for piece in self._plan(m["src_tp"], self.tp):
            if piece.dst_rank != self.rank:
                continue
            pair = self._pair(m["src"], piece.src_rank, "decode")
            buf = torch.empty(self._piece_bytes(piece, m["nblocks"]), dtype=torch.uint8,
                              device=self.kv.device if self.gpu else "cpu")
            works.append([pair.pg.recv([buf], 0, 0), buf, piece, False])
            self.stats["recv_bytes"] += buf.numel()
        self.recvs[m["rid"]] = {"works": works, "blocks": blocks, "m": m, "t0": time.perf_counter()}

    def landed(self) -> list[dict]:
        """Leader: notifications whose receives (on this rank) completed."""
        return [r["m"] for r in self.recvs.values() if all(self._recv_done(w) for w in r["works"])]

    def _recv_done(self, w: list) -> bool:
        # gloo's wait() on a receive waits for the NEXT message each call, so
        # a completed receive must never be waited on again
        if not w[3]:
            w[3] = self._done(w[0])
        return w[3]

    def finish_recv(self, m: dict) -> None:
        """Every decode rank (lockstep): unpack and let the request decode."""
        r = self.recvs.pop(m["rid"], None)
        if r is None:
            return
        for w in r["works"]:
            work, buf, piece, waited = w
            if self.gpu:
                work.wait()  # the compute stream waits for this rank's receive (no host block)
            elif not waited:
                work.wait()
            if r["blocks"] is not None:
                with tracing.span("kv_transfer.unpack"):
                    unpack_blocks(self.kv, buf if self.gpu else buf.to(self.kv.device), r["blocks"],
                                  inner_off=piece.dst_inner_off, inner_bytes=piece.nbytes)
        if r["blocks"] is not None:
            self.engine.finish_remote_prefill(m["rid"], m["tok"], m["lp"])
        self.engine.request_timer.observe_transfer(time.perf_counter() - r["t0"],
                                                   sum(w[1].numel() for w in r["works"]))
        self.stats["recv"] += 1

    def _done(self, work) -> bool:
        if not self.gpu:
            work.wait()
            return True
        return work.is_completed()

    def pending(self) -> int:
        return len(self.sends) + len(self.recvs) + len(self.inbox)


# ------------------------------------------------------------------ wiring
def install_decode(rep, agent: KVTransferAgent) -> None:
    """Every decode rank: handlers for the leader's ext events."""
    rep.handlers["kv_recv"] = agent.post_recv
    rep.handlers["kv_finish"] = agent.finish_recv


def decode_leader_hook(rep, agent: KVTransferAgent):
    """Engine-thread hook on the decode leader: turn notifications and landed
    receives into lockstep ext events."""
    announced: set[str] = set()

    def hook():
        for m in agent.take_notifications():
            rep.submit("kv_recv", m)
        for m in agent.landed():
            if m["rid"] not in announced:
                announced.add(m["rid"])
                rep.submit("kv_finish", m)
        if len(announced) > 4096:  # finished rids no longer pending
            announced.intersection_update(agent.recvs.keys())

    return hook


def install_prefill(rep, agent: KVTransferAgent) -> None:
    """Every prefill rank: send on prefill completion, release the blocks after
    the step (same step on every rank), recycle finished staging buffers."""
    done: list[str] = []
    eng = rep.engine

    def on_prefilled(req) -> None:
        m = req.remote_meta
        bs = eng.kv.block_size
        blocks = req.block_ids[m["skip"]:(len(req.prompt) + bs - 1) // bs]
        agent.send(req.request_id, blocks, m["dst"], req.output[0], req.logprobs[0])
        done.append(req.request_id)

    def after_step() -> None:
        while done:
            eng.finish_transfer(done.pop())
        agent.poll_sends()

    eng.prefill_done_hook = on_prefilled
    rep.post_step_hooks.append(after_step)


def follower_setup(rep, role: str, cp_address: str, engine_id: str, namespace: str, lease_id: int | None) -> None:
    """Runs on TP follower ranks (spawned processes): own control-plane client,
    own transfer endpoint, handlers for the leader's events."""
    from ..runtime.control_plane import SyncControlPlaneClient

    sc = SyncControlPlaneClient(cp_address)
    agent = KVTransferAgent(rep.engine, _CP(sc.client, sc.loop), engine_id, namespace, rep.rank, rep.world)
    agent.start_sync(lease_id)
    rep._kv_agent, rep._cp_client = agent, sc
    if role == "decode":
        install_decode(rep, agent)
    else:
        install_prefill(rep, agent)
