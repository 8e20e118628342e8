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
  P (every rank, lockstep): prefill done -> pack pieces (copy stream, pooled
     staging) -> pg.send; rank 0 publishes notify{rid, src, src_tp, nblocks,
     tok, lp} on `kv_transfer.{ns}.{dst}`; the blocks are released once the
     sends completed.
  D leader: notify -> ext event "kv_recv" -> every decode rank posts its
     receives (same order on every pair); when the leader's receives landed
     -> ext event "kv_finish" -> every rank orders its copy stream after its
     receive, unpacks into the request's blocks, the compute stream waits on
     that unpack's event, finish_remote_prefill -- the same step on every
     rank, so the TP schedulers never diverge.

READ (prefix pull, reference Patch:1296-1360 / worker read RPC 4463-4569):
  P (every rank, scheduler callback, lockstep): the decode worker caches more
     of the prompt than this worker -> rank 0 publishes read{rid, src, src_tp,
     first, last} to the decode engine; every rank posts receives for the
     pieces of blocks [first, last) addressed to it on the reverse-direction
     pair group; when the leader's receives landed -> ext event
     "kv_read_done" -> every rank unpacks and the scheduler computes only the
     rest of the prompt.
  D leader: read -> ext event "kv_read" -> every decode rank packs its pieces
     of the request's cached blocks and sends them (reverse group).
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
from .transfer import StagingPool, pack_blocks, tp_relayout_plan, unpack_blocks

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
        self.reads: dict[str, dict] = {}  # prefill side: prefix pulls in flight (same shape)
        self.served: collections.deque = collections.deque()  # decode side: (work, buf) of served reads
        self.stats = dict(sent=0, recv=0, sent_bytes=0, recv_bytes=0, reads=0, read_bytes=0, served=0)
        self.copy_stream = torch.cuda.Stream(self.kv.device) if self.gpu else None
        self.pool = StagingPool(self.kv.device if self.gpu else "cpu")
        self._retiring: collections.deque = collections.deque()  # (event, [bufs]) until unpacks finish

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

    def _pair(self, peer: str, peer_rank: int, role: str, rev: bool = False) -> _Pair:
        """role 'prefill': I am rank 0 of the pair and connect to the peer's
        (decode) store.  rev: the decode -> prefill group of the pair (READ
        traffic gets its own communicator, so the two directions never share
        an in-order RCCL stream)."""
        key = (role, peer, peer_rank, rev)
        p = self.pairs.get(key)
        if p is not None:
            return p
        if role == "prefill":
            m = self._meta(peer, peer_rank)
            store = dist.TCPStore(m["host"], m["port"], is_master=False, timeout=datetime.timedelta(seconds=120))
            prefix = f"{'rev' if rev else ''}pair/{self.engine_id}.{self.rank}/{peer}.{peer_rank}"
            rank = 0
        else:
            store = self.store
            prefix = f"{'rev' if rev else ''}pair/{peer}.{peer_rank}/{self.engine_id}.{self.rank}"
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
            self._sync_copy_stream()
            for piece in self._plan(self.tp, dst_tp):
                if piece.src_rank != self.rank:
                    continue
                pair = self._pair(dst_engine, piece.dst_rank, "prefill")
                base = self.pool.take(self._piece_bytes(piece, len(block_ids)))
                with self._on_copy_stream():
                    buf = pack_blocks(self.kv, block_ids, inner_off=piece.src_inner_off, inner_bytes=piece.nbytes,
                                      out=base[:self._piece_bytes(piece, len(block_ids))])
                    work = pair.pg.send([buf], 1, 0)
                self.sends.append((rid, work, base))
                self.stats["sent_bytes"] += buf.numel()
        self.stats["sent"] += 1

    def poll_sends(self) -> int:
        """Recycle staging buffers of completed sends; returns how many are still in flight."""
        while self.sends and self._done(self.sends[0][1]):
            self.pool.give(self.sends.popleft()[2])
        self._retire()
        return len(self.sends)

    # --------------------------------------------------------------- streams / staging
    def _on_copy_stream(self):
        return torch.cuda.stream(self.copy_stream) if self.copy_stream is not None else _Null()

    def _sync_copy_stream(self) -> None:
        """The copy stream sees everything the compute stream enqueued so far
        (the prefill forward that wrote the blocks being packed)."""
        if self.copy_stream is not None:
            self.copy_stream.wait_stream(torch.cuda.current_stream(self.kv.device))

    def _after_copy(self, bufs: list) -> None:
        """The compute stream waits for the unpacks just enqueued on the copy
        stream (GPU-side, no host block); the staging goes back to the pool
        once they finished."""
        if self.copy_stream is not None:
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            torch.cuda.current_stream(self.kv.device).wait_event(ev)
            self._retiring.append((ev, bufs))
        else:
            for b in bufs:
                self.pool.give(b)

    def _retire(self) -> None:
        while self._retiring and self._retiring[0][0].query():
            for b in self._retiring.popleft()[1]:
                self.pool.give(b)

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
            n = self._piece_bytes(piece, m["nblocks"])
            base = self.pool.take(n)
            works.append([pair.pg.recv([base[:n]], 0, 0), base[:n], piece, False, base])
            self.stats["recv_bytes"] += n
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
        self._unpack_all(r)
        if r["blocks"] is not None:
            self.engine.finish_remote_prefill(m["rid"], m["tok"], m["lp"])
        self.engine.request_timer.observe_transfer(time.perf_counter() - r["t0"],
                                                   sum(w[1].numel() for w in r["works"]))
        self.stats["recv"] += 1

    def _unpack_all(self, r: dict) -> None:
        with self._on_copy_stream(), tracing.span("kv_transfer.unpack"):
            for w in r["works"]:
                work, buf, piece, waited = w[:4]
                if self.gpu:
                    work.wait()  # the copy stream waits for this rank's receive (no host block)
                elif not waited:
                    work.wait()
                if r["blocks"] is not None:
                    unpack_blocks(self.kv, buf if self.gpu else buf.to(self.kv.device), r["blocks"],
                                  inner_off=piece.dst_inner_off, inner_bytes=piece.nbytes)
        self._after_copy([w[4] for w in r["works"]])

    # --------------------------------------------------------------- READ: prefill side
    def request_read(self, req, first: int, last: int, dst_engine: str) -> None:
        """Every prefill rank (scheduler callback, lockstep): pull blocks
        [first, last) of the prompt from the decode engine's cache."""
        src_tp = self._meta(dst_engine, 0)["tp"]
        rid = req.request_id
        if self.rank == 0:
            note = msgpack.packb({"t": "read", "rid": rid, "src": self.engine_id, "src_tp": self.tp,
                                  "first": first, "last": last})
            self.cp.fire("publish", f"kv_transfer.{self.ns}.{dst_engine}", note)
        works = []
        for piece in self._plan(src_tp, self.tp):  # decode ranks -> prefill ranks
            if piece.dst_rank != self.rank:
                continue
            pair = self._pair(dst_engine, piece.src_rank, "prefill", rev=True)
            n = self._piece_bytes(piece, last - first)
            base = self.pool.take(n)
            works.append([pair.pg.recv([base[:n]], 1, 0), base[:n], piece, False, base])
            self.stats["read_bytes"] += n
        self.reads[rid] = {"works": works, "blocks": list(req.block_ids[first:last]), "m": {"rid": rid}}
        self.stats["reads"] += 1

    def reads_landed(self) -> list[str]:
        """Leader: pulls whose receives (on this rank) completed."""
        return [rid for rid, r in self.reads.items() if all(self._recv_done(w) for w in r["works"])]

    def finish_read(self, rid: str) -> None:
        """Every prefill rank (lockstep): unpack the pulled prefix, resume the request."""
        r = self.reads.pop(rid, None)
        if r is None:
            return
        self._unpack_all(r)
        self.engine.finish_remote_read(rid)

    # --------------------------------------------------------------- READ: decode side
    def serve_read(self, m: dict) -> None:
        """Every decode rank (lockstep): send this rank's pieces of the
        request's cached blocks [first, last) to the pulling prefill engine."""
        req = self.engine.scheduler.remote.get(m["rid"])
        n_blocks = m["last"] - m["first"]
        blocks = req.block_ids[m["first"]:m["last"]] if req is not None else [0] * n_blocks  # gone: any bytes
        self._sync_copy_stream()
        for piece in self._plan(self.tp, m["src_tp"]):
            if piece.src_rank != self.rank:
                continue
            pair = self._pair(m["src"], piece.dst_rank, "decode", rev=True)
            n = self._piece_bytes(piece, n_blocks)
            base = self.pool.take(n)
            with self._on_copy_stream():
                buf = pack_blocks(self.kv, blocks, inner_off=piece.src_inner_off, inner_bytes=piece.nbytes,
                                  out=base[:n])
                self.served.append((pair.pg.send([buf], 0, 0), base))
        self.stats["served"] += 1

    def poll_served(self) -> int:
        while self.served and self._done(self.served[0][0]):
            self.pool.give(self.served.popleft()[1])
        self._retire()
        return len(self.served)

    def _done(self, work) -> bool:
        if not self.gpu:
            work.wait()
            return True
        return work.is_completed()

    def pending(self) -> int:
        return len(self.sends) + len(self.recvs) + len(self.inbox) + len(self.reads) + len(self.served)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


# ------------------------------------------------------------------ wiring
def install_decode(rep, agent: KVTransferAgent) -> None:
    """Every decode rank: handlers for the leader's ext events."""
    rep.handlers["kv_recv"] = agent.post_recv
    rep.handlers["kv_finish"] = agent.finish_recv
    rep.handlers["kv_read"] = agent.serve_read
    rep.post_step_hooks.append(agent.poll_served)


def decode_leader_hook(rep, agent: KVTransferAgent):
    """Engine-thread hook on the decode leader: turn notifications and landed
    receives into lockstep ext events."""
    announced: set[str] = set()

    def hook():
        for m in agent.take_notifications():
            rep.submit("kv_read" if m.get("t") == "read" else "kv_recv", m)
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
        agent.poll_sends()
        # blocks go back to the pool only after their sends completed (the
        # send reads the staging copy; the pack reads the blocks)
        sent = {s[0] for s in agent.sends}
        for rid in [r for r in done if r not in sent]:
            done.remove(rid)
            eng.finish_transfer(rid)

    def on_read(req, first: int, last: int) -> None:
        agent.request_read(req, first, last, req.remote_meta["dst"])

    eng.prefill_done_hook = on_prefilled
    eng.scheduler.on_remote_read = on_read
    rep.handlers["kv_read_done"] = agent.finish_read
    rep.post_step_hooks.append(after_step)


def prefill_leader_hook(rep, agent: KVTransferAgent):
    """Engine-thread hook on the prefill leader: landed prefix pulls become
    lockstep "kv_read_done" events."""
    announced: set[str] = set()

    def hook():
        for rid in agent.reads_landed():
            if rid not in announced:
                announced.add(rid)
                rep.submit("kv_read_done", rid)
        if len(announced) > 4096:
            announced.intersection_update(agent.reads.keys())

    return hook


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
