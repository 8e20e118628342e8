"""KV transfer agent: the control-plane shell around the data plane
(`transfer.KVDataPlane`), per TP rank -- the reference's NIXL connector +
NixlMetadataStore + per-rank notification counting (SURVEY §2.6 V3-V7, G8;
Patch:1296-1424, :2991, :3252-3255).

The same agent runs in the `dynamo serve` prefill / decode workers
(llm/workers.py) and in the headline benchmark (disagg/bench_disagg.py); they
differ only in how ranks reach each other:

* `StoreLinks` (serving, default): every rank hosts a c10d TCPStore and
  publishes `{ns}/kv_transfer/{engine_id}/{rank}` (lease-bound) with its
  address and the engine's TP size; a (prefill rank, decode rank) pair gets
  its own 2-rank process group on a PrefixStore of the decode rank's store
  (ProcessGroupNCCL = RCCL over xGMI on GPUs, gloo on CPU), one per
  direction, created at the first transfer -- workers join and leave without
  any global communicator rebuild.
* `transfer.WorldLinks` (bench): the ranks of one torch.distributed world.

Transport (`kv_transport`, the workers' `--kv-transport`; never implicit):
"rccl" (default on GPUs) moves device staging buffers over per-pair RCCL
communicators, which need the two ranks on distinct GPUs; "host" stages KV
through pinned host memory over per-pair gloo groups, so a prefill and a
decode worker may share ONE GPU (functional tests of the served graph on a
one-GPU box).  Both ends publish their transport; a mismatch is refused.
"ipc" is the one-sided WRITE (NIXL-like, Patch:1361-1424): every decode rank
shares its KV cache (VMM chunks whose dma-buf fds it serves on a Unix socket,
kv_share.py), the prefill rank maps it and writes
each layer group straight into the request's decode blocks from its copy
stream -- no staging, no receive kernel, no RCCL kernel that could hold a
hardware queue, and it works between two processes on ONE GPU too.  The
decode engine learns the bytes landed from "done", which the prefill leader
publishes only after the copy stream passed the request's last write.
Prefill TP 1 only (one writer per request; the decode side may be TP > 1).
The prefix READ over it is one-sided too: "read1" asks the decode engine to
pin the cached blocks and name them ("read1_ok"), the prefill rank copies
them out of the mapped decode caches into its own blocks, and "read1_done"
unpins them; both ends hold the blocks (read_pinned / write_pending) while
the copy may run.

Notifications are published by the engine leader (TP rank 0) only; every
data-plane call runs on every rank in lockstep, driven by the engine's own
schedule or by ReplicatedEngine extension events (parallel/tp.py).  Two
channels:

* `kv_wire.{ns}` (one subject for the whole namespace): the messages that
  make ranks enqueue RCCL work -- a prefill forward's announcements (ONE
  "start" message per forward, entries for every destination engine) and
  prefix "read" requests -- plus "cancel".
* `kv_transfer.{ns}.{engine}`: "done", "fail", "read_verdict".

Deadlock freedom of the RCCL wire (`WireOrder`).  An RCCL send / recv kernel
holds its stream's hardware queue until the peer's matching kernel runs, and
ROCm maps all of a process's RCCL streams onto a few queues (utils/streams.py),
so two transfers enqueued in opposite orders on two ranks can wait on each
other -- e.g. a prefill rank's READ receive ahead of its WRITE send while the
decode rank has the WRITE receive ahead of the READ send.
The control plane is one server that delivers a subject's messages in one
order, which is a total order of all wire messages.  Every rank enqueues its
RCCL work in that order: a prefill rank publishes a message and enqueues its
ops before publishing the next (program order on one connection), a decode
rank posts the ops of the messages addressed to it in arrival order from ONE
FIFO (staging backpressure stalls the FIFO head, it never lets a later
message overtake).  Then the wire op with the smallest key still pending is
at the front of both of its ranks' queues whatever the queue sharing, so it
completes; by induction every op does.  The reference avoids the same hazard
with a per-transfer rendezvous (Patch:2568-2613, "PUT" before NCCL send).

WRITE, layer-streamed, per request of a prefill batch:
  P (all ranks) batch_hook, before the forward: begin_send (staging taken
     against the admission reservation); leader publishes ONE
     start{src, src_tp, by_dst{engine: [rid, nblocks]}} on the wire subject.
  P (all ranks) layer hook: pack + send each finished layer group's pieces;
     after the step: end_forward; on the first token (prefill_done_hook) the
     leader publishes done{rid, tok, lp} and the request's blocks are
     released at the same step on every rank.
  D leader: start -> (when its staging pool can take the bytes, in wire
     order) ext "kv_recv" -> every rank posts its receives; when done
     arrived and the leader's receives landed -> ext "kv_finish" -> every rank
     unpacks (skipped, drain only, if the request was cancelled meanwhile)
     and the request joins the decode batch.
READ (prefix pull):
  P (all ranks) scheduler callback: leader publishes read{rid, dst, src,
     src_tp, first, last} on the wire subject; every rank posts its
     reverse-direction receives; when the leader's landed AND the decode
     engine's read_verdict arrived -> ext "kv_read_done" -> every rank unpacks
     (drain only if the request is no longer READING or the verdict is
     false) and the scheduler resumes it (recomputing the prefix on false).
  D leader: read -> (staging permitting, in wire order) ext "kv_read" ->
     every rank packs and sends its pieces of the cached blocks; the verdict
     says whether they were the request's blocks (a READ that
     arrives after the decode engine gave the request up gets filler bytes
     and verdict false, so the prefill engine never registers them).
Cancel: a decode engine that falls back to a local prefill publishes cancel
  {rid}; a prefill engine skips the request if it has not taken it yet.
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
from .transfer import KVDataPlane, RemoteKV

log = logging.getLogger("dynamo_exp_amd.disagg.agent")

META_PREFIX = "kv_transfer/"

# one-sided transport, peers in THIS process (tests, the loopback 1P1D):
# (engine id, rank) -> KV cache tensor, used instead of an IPC mapping
LOCAL_KV: dict[tuple, torch.Tensor] = {}


class _CP:
    """Blocking control-plane calls from a non-event-loop thread."""

    def __init__(self, client, loop: asyncio.AbstractEventLoop):
        self.client, self.loop = client, loop

    def call(self, name: str, *a, **kw):
        return asyncio.run_coroutine_threadsafe(getattr(self.client, name)(*a, **kw), self.loop).result(30)

    def fire(self, name: str, *a, **kw) -> None:
        asyncio.run_coroutine_threadsafe(getattr(self.client, name)(*a, **kw), self.loop)


class StoreLinks:
    """Per-pair process groups on the decode rank's TCPStore (serving)."""

    def __init__(self, agent: "KVTransferAgent"):
        self.agent = agent
        self.pairs: dict[tuple, tuple] = {}

    def _pair(self, peer: str, peer_rank: int, prefill_side: bool, rev: bool):
        """The pair's process group and my rank in it (prefill side = 0).
        rev: the decode -> prefill group (READ traffic has its own
        communicator)."""
        key = (peer, peer_rank, prefill_side, rev)
        p = self.pairs.get(key)
        if p is not None:
            return p
        a = self.agent
        tag = "rev" if rev else ""
        if prefill_side:
            m = a.meta_of(peer, peer_rank)
            store = dist.TCPStore(m["host"], m["port"], is_master=False, timeout=datetime.timedelta(seconds=120))
            prefix = f"{tag}pair/{a.engine_id}.{a.rank}/{peer}.{peer_rank}"
            rank = 0
        else:
            store = a.store
            prefix = f"{tag}pair/{peer}.{peer_rank}/{a.engine_id}.{a.rank}"
            rank = 1
        ps = dist.PrefixStore(prefix, store)
        timeout = datetime.timedelta(seconds=300)
        if a.transport == "rccl":
            pg = dist.ProcessGroupNCCL(ps, rank, 2, timeout)
        else:
            pg = dist.ProcessGroupGloo(ps, rank, 2, timeout)
        p = self.pairs[key] = (pg, rank)
        return p

    def send(self, engine: str, rank: int, t: torch.Tensor, rev: bool = False):
        pg, me = self._pair(engine, rank, prefill_side=not rev, rev=rev)
        return pg.send([t], 1 - me, 0)

    def recv(self, engine: str, rank: int, t: torch.Tensor, rev: bool = False):
        pg, me = self._pair(engine, rank, prefill_side=rev, rev=rev)
        return pg.recv([t], 1 - me, 0)


class KVTransferAgent:
    """One TP rank's KV transfer endpoint.  `engine` is the rank's LLMEngine;
    `cp` a blocking control-plane handle (`_CP`); `links` defaults to
    StoreLinks (serving); the bench passes transfer.WorldLinks."""

    def __init__(self, engine, cp: _CP, engine_id: str, namespace: str = "dynamo", tp_rank: int = 0,
                 tp_size: int = 1, host: str | None = None, links=None, host_staging: bool = False,
                 pool_cap_bytes: int | None = None, layer_group_count: int = 4, kv_transport: str | None = None):
        self.engine = engine
        engine.kv_transfer_attached = True  # its kv_scales are now published: calibrate_kv_scales refuses
        self.cp = cp
        self.engine_id = engine_id
        self.ns = namespace
        self.rank, self.tp = tp_rank, tp_size
        self.kv = engine.runner.kv_cache
        self.gpu = self.kv.is_cuda
        if kv_transport not in (None, "rccl", "host", "ipc"):
            raise ValueError(f"kv_transport {kv_transport!r}: expected 'rccl', 'host' or 'ipc'")
        one_sided = kv_transport == "ipc"
        host_staging = (host_staging or kv_transport == "host") and self.gpu and not one_sided
        # what the bytes ride on: RCCL between distinct GPUs, gloo for host-staged / CPU engines,
        # or the one-sided WRITE through the decode cache's IPC mapping
        self.transport = ("ipc" if one_sided else
                          "rccl" if (self.gpu and not host_staging) else ("host" if self.gpu else "gloo"))
        self._ipc_maps: dict[tuple, RemoteKV] = {}
        self._ipc_owned: list = []
        self._ipc_by_key: dict[tuple, object] = {}  # (engine, rank) -> RemoteMapping
        self._done_wait: dict[str, tuple] = {}  # one-sided, leader: rid -> (dst, done msg) until the write landed
        self._write_dst: dict[str, str] = {}  # one-sided: rid -> decode engine, writes in flight
        self._written: set[str] = set()  # one-sided: writes landed, "done" / "fail" not yet published
        self._read1: dict[str, tuple] = {}  # one-sided READ, prefill: rid -> (decode engine, my blocks, its TP)
        self._read1_t0: dict[str, float] = {}  # leader: when each one-sided READ was asked
        self._unmapped: set[str] = set()  # one-sided: requests whose decode cache could not be mapped
        self._write_t0: dict[str, tuple] = {}  # one-sided, decode: rid -> (start time, bytes written)
        if one_sided:
            LOCAL_KV[(engine_id, tp_rank)] = self.kv
        self.host = host or os.environ.get("DX_HOST_IP", "127.0.0.1")
        self.store = None
        if links is None:
            self.store = dist.TCPStore(self.host, 0, is_master=True, wait_for_workers=False,
                                       timeout=datetime.timedelta(seconds=120))
            links = StoreLinks(self)
        cap = pool_cap_bytes or int(os.environ.get("DX_KV_STAGING_BYTES", str(4 << 30)))
        self.dp = KVDataPlane(self.kv, links, tp_rank, tp_size, engine.model.cfg.num_key_value_heads,
                              host_staging=host_staging, layer_group_count=layer_group_count, pool_cap_bytes=cap,
                              one_sided=one_sided, remote_kv=self._remote_kv if one_sided else None)
        self.meta_cache: dict[tuple, dict] = {}
        self.tp_cache: dict[str, int] = {}  # engine id -> TP size (from requests or metadata)
        self.inbox: collections.deque = collections.deque()  # leader: notifications
        self.stats = dict(sent=0, recv=0, reads=0, served=0, deferred=0)
        self.reservations: dict[str, int] = {}  # leader, prefill side: rid -> reserved staging bytes
        # decode leader: per-request transfer milestones (perf_counter), when a
        # caller sets record_spans (bench.py N > 1): enq (prefill queued), start
        # (the prefill forward announced it), posted (receives posted), landed,
        # done (first token arrived), joined (unpacked, decoding)
        self.record_spans = False
        self.spans: dict[str, dict] = {}
        # request ids decode engines gave up on (wire "cancel"), bounded; and,
        # prefill leader, the decode engines' verdicts on served READs
        self.cancelled: collections.OrderedDict = collections.OrderedDict()
        self.read_verdicts: dict[str, bool] = {}
        self.cancel_seq = 0

    @property
    def pool(self):
        return self.dp.pool

    def span(self, rid: str, what: str) -> None:
        if self.record_spans:
            self.spans.setdefault(rid, {}).setdefault(what, time.perf_counter())

    def span_summary(self) -> dict:
        """p50 / p90 / mean ms of the transfer phases over the recorded requests:
        queue (enq -> start: prefill queue + batching), forward_to_landed
        (start -> landed: the layer-streamed WRITE riding the prefill forward),
        landed_to_joined (landed / first token -> decoding), total (enq -> joined)."""
        def stats(xs):
            if not xs:
                return None
            xs = sorted(xs)
            return {"p50": round(xs[len(xs) // 2] * 1e3, 2), "p90": round(xs[int(len(xs) * 0.9)] * 1e3, 2),
                    "mean": round(sum(xs) / len(xs) * 1e3, 2), "n": len(xs)}

        sp = [v for v in self.spans.values() if "joined" in v and "enq" in v and "start" in v]
        out = {"queue": stats([v["start"] - v["enq"] for v in sp]),
               "forward_to_landed": stats([v["landed"] - v["start"] for v in sp if "landed" in v]),
               "landed_to_joined": stats([v["joined"] - max(v.get("landed", 0), v.get("done", 0)) for v in sp]),
               "total": stats([v["joined"] - v["enq"] for v in sp])}
        return out

    # --------------------------------------------------------------- metadata
    @property
    def meta_key(self) -> str:
        return f"{self.ns}/{META_PREFIX}{self.engine_id}/{self.rank}"

    def meta(self) -> bytes:
        lay = self.dp.lay
        m = {"engine_id": self.engine_id, "rank": self.rank, "tp": self.tp, "host": self.host,
             "port": self.store.port if self.store is not None else None,
             "backend": "nccl" if self.transport == "rccl" else "gloo",
             "transport": self.transport, "kv_dtype": str(self.dp.kv.dtype),
             "kv_scales": self.kv_scales(),
             "kv_layout": [lay.num_layers, lay.num_blocks, lay.block_bytes]}
        share = getattr(self.engine.runner, "kv_share", None)
        if self.transport == "ipc" and self.gpu and share is not None:
            # the cache's chunk fds, served on a Unix socket (kv_share.py; not
            # hipIpcGetMemHandle: imports of allocations over ~1 GiB never return)
            m["kv_share"] = [share.serve(f"{self.engine_id}-{self.rank}"), self.kv.data_ptr() - share.ptr]
        return json.dumps(m).encode()

    def _remote_kv(self, engine_id: str, rank: int) -> RemoteKV:
        """One-sided transport: a decode rank's KV cache -- the tensor itself
        for a peer in this process, else its IPC mapping (opened once, kept
        until close())."""
        key = (engine_id, rank)
        r = self._ipc_maps.get(key)
        if r is not None:
            return r
        m = self.meta_of(engine_id, rank)
        L, nb, bb = m["kv_layout"]
        t = LOCAL_KV.get(key)
        if t is not None:
            r = RemoteKV(nb, bb, L, tensor=t)
        elif "kv_share" in m and self.gpu:
            from .kv_share import RemoteMapping

            addr, off = m["kv_share"]
            mp_ = RemoteMapping(addr, self.kv.device)
            self._ipc_owned.append(mp_)
            self._ipc_by_key[key] = mp_
            if off + L * 2 * nb * bb > mp_.total:
                raise RuntimeError(f"engine {engine_id} rank {rank}: its KV layout does not fit its shared buffer")
            r = RemoteKV(nb, bb, L, ptr=mp_.ptr + off)
        else:
            raise RuntimeError(f"one-sided KV transport: engine {engine_id} rank {rank} is neither in this "
                               "process nor sharing its KV cache (a decode engine needs kv_shared=True)")
        self._ipc_maps[key] = r
        return r

    def engine_gone(self, engine_id: str) -> bool:
        """Whether an engine's transfer metadata (lease-bound) has disappeared."""
        if self.cp is None:
            return False
        return self.cp.call("get", f"{self.ns}/{META_PREFIX}{engine_id}/0") is None

    def gc_peers(self) -> int:
        """One-sided transport, prefill side: unmap the KV caches of decode
        engines whose transfer metadata is gone (lease expired: the worker
        left or died) once no write to them is in flight -- a mapping keeps
        the dead worker's device memory allocated.  Returns how many were
        unmapped."""
        busy = {x.peer for x in self.dp.sends.values()}
        n = 0
        for key in list(self._ipc_by_key):
            engine_id, rank = key
            if engine_id in busy:
                continue
            if self.cp.call("get", f"{self.ns}/{META_PREFIX}{engine_id}/{rank}") is not None:
                continue
            mp_ = self._ipc_by_key.pop(key)
            self._ipc_maps.pop(key, None)
            self.meta_cache.pop(key, None)
            if self.gpu:
                torch.cuda.synchronize(self.kv.device)
            mp_.close()
            self._ipc_owned.remove(mp_)
            n += 1
            log.info("unmapped the KV cache of departed engine %s rank %d", engine_id, rank)
        return n

    def close(self) -> None:
        """Unmap the peers' KV caches (one-sided transport), after this
        rank's writes drained."""
        if self._ipc_owned:
            if self.gpu:
                torch.cuda.synchronize(self.kv.device)
            for mp_ in self._ipc_owned:
                mp_.close()
        self._ipc_owned, self._ipc_maps, self._ipc_by_key = [], {}, {}
        if LOCAL_KV.get((self.engine_id, self.rank)) is self.kv:
            del LOCAL_KV[(self.engine_id, self.rank)]

    def kv_scales(self) -> list[float]:
        """Per-tensor (K, V) scales of this engine's KV bytes (fp8 caches;
        (1, 1) for bf16): raw e4m3 bytes only mean the same values on two
        engines whose scales agree."""
        return [float(x) for x in getattr(self.engine.model, "kv_scales", (1.0, 1.0))]

    @property
    def subject(self) -> str:
        return f"kv_transfer.{self.ns}.{self.engine_id}"

    @property
    def wire_subject(self) -> str:
        """The namespace's one ordered channel of RCCL-enqueuing messages
        (module docstring: deadlock freedom)."""
        return f"kv_wire.{self.ns}"

    def _on_wire(self, m: dict) -> None:
        """Pump thread: keep the wire messages addressed to this engine, in
        arrival order, in the same inbox as the direct notifications."""
        t = m.get("t")
        if t == "cancel":
            self.cancelled[m["rid"]] = True
            self.cancel_seq += 1
            while len(self.cancelled) > 65536:
                self.cancelled.popitem(last=False)
        elif t == "start":
            reqs = m["by_dst"].get(self.engine_id)
            if reqs:
                self.inbox.append({"t": "start", "src": m["src"], "src_tp": m["src_tp"], "reqs": reqs})
        elif t == "read" and m.get("dst") == self.engine_id:
            self.inbox.append(m)

    async def start_async(self, cp_async, lease_id: int | None = None) -> "KVTransferAgent":
        """Leader (rank 0), inside an event loop: publish metadata and listen
        for notifications addressed to this engine and for the wire channel."""
        await cp_async.put(self.meta_key, self.meta(), lease=lease_id)
        sub = await cp_async.subscribe(self.subject)
        wire = await cp_async.subscribe(self.wire_subject)

        async def pump():
            async for item in sub:
                self.inbox.append(msgpack.unpackb(item["data"], raw=False))

        async def pump_wire():
            async for item in wire:
                self._on_wire(msgpack.unpackb(item["data"], raw=False))

        self._sub_task = asyncio.create_task(pump())
        self._wire_task = asyncio.create_task(pump_wire())
        return self

    def is_cancelled(self, rid: str) -> bool:
        return rid in self.cancelled

    def start_sync(self, lease_id: int | None = None) -> "KVTransferAgent":
        """Followers: publish metadata only (notifications reach the leader)."""
        self.cp.call("put", self.meta_key, self.meta(), lease=lease_id)
        return self

    def meta_of(self, engine_id: str, rank: int = 0) -> dict:
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
            m = json.loads(raw)
            if m.get("transport", self.transport) != self.transport:
                raise RuntimeError(f"engine {engine_id} moves KV over {m['transport']}, this one over "
                                   f"{self.transport}: prefill and decode workers need the same --kv-transport")
            mine = str(self.dp.kv.dtype)
            if m.get("kv_dtype", mine) != mine:  # raw KV bytes only mean the same thing in one dtype
                raise RuntimeError(f"engine {engine_id} has a {m['kv_dtype']} KV cache, this one {mine}: "
                                   "prefill and decode workers need the same kv_cache_dtype")
            theirs, ours = m.get("kv_scales"), self.kv_scales()
            if theirs is not None and any(abs(a - b) > 1e-6 * max(1.0, abs(b)) for a, b in zip(theirs, ours)):
                raise RuntimeError(f"engine {engine_id} quantises its KV with scales {theirs}, this one {ours}: "
                                   "prefill and decode workers need the same kv_scales (calibrate once, "
                                   "pass the result to every worker)")
            self.meta_cache[key] = m
        return m

    def tp_of(self, engine_id: str) -> int:
        tp = self.tp_cache.get(engine_id)
        if tp is None:
            tp = self.tp_cache[engine_id] = int(self.meta_of(engine_id, 0)["tp"])
        return tp

    def _publish(self, engine_id: str, msg: dict) -> None:
        if self.rank == 0 and self.cp is not None:  # (cp None: an agent without a control plane, tests)
            self.cp.fire("publish", f"kv_transfer.{self.ns}.{engine_id}", msgpack.packb(msg))

    def _publish_wire(self, msg: dict) -> None:
        """Leader: a message on the ordered wire channel.  `cp.fire` hands
        publishes to the event loop in call order and the client writes them
        under a FIFO lock on one connection, so they reach the server in
        program order; every rank enqueues the RCCL work a message announces
        after this call and before the next wire message, which is all the
        order argument (module docstring) needs."""
        if self.rank == 0 and self.cp is not None:
            self.cp.fire("publish", self.wire_subject, msgpack.packb(msg))

    # --------------------------------------------------------------- prefill side
    def admit(self, rid: str, nblocks: int, read_blocks: int, dst_engine: str) -> bool:
        """Leader, before adding a dequeued request: reserve the staging its
        WRITE (and prefix READ) will take; False = not now (backpressure)."""
        dst_tp = self.tp_of(dst_engine)
        if self.dp.one_sided:  # no staging: the reservation only tracks whether the WRITE started
            self.reservations[rid] = [0, 0, False, dst_engine, True]
            return True
        ns = self.dp.send_bytes(nblocks, dst_tp)
        nr = self.dp.recv_bytes(read_blocks, dst_tp) if read_blocks else 0
        if not self.pool.reserve(ns, nr):
            self.stats["deferred"] += 1
            return False
        # [send bytes, read bytes, seen in the engine, decode engine, WRITE not started yet]
        self.reservations[rid] = [ns, nr, False, dst_engine, True]
        return True

    def remote_meta(self, r, read_blocks: int) -> dict:
        """The prefill engine's remote_meta of a dequeued RemotePrefillRequest
        (serving worker, bench, loopback)."""
        m = {"dst": r.engine_id, "dst_tp": r.engine_tp or None, "skip": r.skip_blocks, "read_blocks": read_blocks}
        if self.dp.one_sided:
            m["dst_blocks"] = list(r.block_ids)
        return m

    def _release_reservation(self, rid: str) -> None:
        """Give back whatever is left of a request's reservation (its READ
        was skipped because the local prefix cache covered it, or it left the
        engine before using it)."""
        r = self.reservations.pop(rid, None)
        if r is not None:
            self.pool.unreserve(r[0])
            self.pool.unreserve(r[1])

    def gc_reservations(self) -> None:
        """Leader, after each step: a request seen in the engine that is now
        gone (aborted, finished) releases the rest of its reservation."""
        reqs = self.engine.requests
        for rid, r in list(self.reservations.items()):
            if rid in reqs:
                r[2] = True
            elif r[2]:
                if r[4]:  # its WRITE never started: the decode worker prefills it itself
                    self._publish(r[3], {"t": "fail", "rid": rid})
                    self.stats["failed"] = self.stats.get("failed", 0) + 1
                self._release_reservation(rid)

    def _use_reservation(self, rid: str, part: int) -> None:
        """The leader is about to take the staging of a reserved part
        (0 = send, 1 = read): release that share of the reservation first."""
        r = self.reservations.get(rid)
        if r is not None:
            self.pool.unreserve(r[part])
            r[part] = 0
            if part == 0:
                r[4] = False
            if not (r[0] or r[1] or r[4]):
                del self.reservations[rid]

    def on_batch(self, batch) -> None:
        """Every prefill rank, before the forward: announce the remote-decode
        requests whose prompt this batch completes."""
        bs = self.dp.block_size
        anns: dict[str, list] = {}
        for r, smp in zip(batch.requests[:batch.n_prefill], batch.sample):
            if not (smp and r.remote_decode):
                continue
            m = r.remote_meta
            dst = m["dst"]
            dst_tp = int(m.get("dst_tp") or self.tp_of(dst))
            skip = m.get("skip", 0)
            blocks = r.block_ids[skip:(len(r.prompt) + bs - 1) // bs]
            dst_blocks = None
            if self.dp.one_sided:
                if self.tp != 1:
                    raise RuntimeError("the one-sided (ipc) KV transport needs prefill TP 1")
                if "dst_blocks" not in m:
                    raise RuntimeError(f"one-sided WRITE of {r.request_id}: remote_meta has no dst_blocks")
                dst_blocks = m["dst_blocks"][skip:skip + len(blocks)]
                try:  # map the decode caches now, not inside the forward's layer hooks
                    for pc in self.dp._my(self.tp, dst_tp, "src"):
                        self._remote_kv(dst, pc.dst_rank)
                except Exception as e:  # noqa: BLE001 -- the decode worker is gone or unreachable
                    log.warning("one-sided WRITE of %s: cannot map %s's KV cache (%s): the decode worker "
                                "prefills it itself", r.request_id, dst, e)
                    self._unmapped.add(r.request_id)
                    self._use_reservation(r.request_id, 0)
                    self._release_reservation(r.request_id)
                    self._publish(dst, {"t": "fail", "rid": r.request_id})
                    continue
                self._write_dst[r.request_id] = dst
            self._use_reservation(r.request_id, 0)
            # a READ happens before any of the prompt is computed: whatever
            # is still reserved for it now (pull skipped) is not needed
            self._release_reservation(r.request_id)
            anns.setdefault(dst, []).append(self.dp.begin_send(r.request_id, blocks, dst, dst_tp, dst_blocks))
        if anns:  # ONE wire message per forward, whatever the destinations
            self._publish_wire({"t": "start", "src": self.engine_id, "src_tp": self.tp, "by_dst": anns})

    def on_prefilled(self, req) -> None:
        """Every prefill rank, first token sampled: the leader tells the
        decode engine; the blocks are released after this step (the bytes
        are in staging: end_forward ordered the compute stream after the packs)."""
        FAULTS.before_kv_transfer_sync()
        msg = {"t": "done", "rid": req.request_id, "tok": req.output[0], "lp": req.logprobs[0]}
        if req.request_id in self._unmapped:  # its WRITE never started ("fail" went out in on_batch)
            self._unmapped.discard(req.request_id)
            self._released.append(req.request_id)
            return
        if self.dp.one_sided:  # the decode engine reads its blocks on "done": publish once the writes landed
            self._done_wait[req.request_id] = (req.remote_meta["dst"], msg)
            if req.request_id in self._written:
                self.poll_sends()
        else:
            self._publish(req.remote_meta["dst"], msg)
        self._released.append(req.request_id)
        self.stats["sent"] += 1

    def on_read(self, req, first: int, last: int) -> None:
        """Every prefill rank (scheduler callback): pull blocks [first, last)
        of the prompt from the decode engine's cache."""
        m = req.remote_meta
        dst = m["dst"]
        src_tp = int(m.get("dst_tp") or self.tp_of(dst))
        if self.dp.one_sided:
            # one-sided READ: ask the decode engine to pin the blocks and name
            # them ("read1" -> "read1_ok"), copy them from its mapped cache
            # (kv_read1_go), unpin ("read1_done"); the request's own blocks are
            # held (write_pending) until the copy landed
            rid = req.request_id
            self.engine.scheduler.write_pending.add(rid)
            self._read1[rid] = (dst, list(req.block_ids[first:last]), src_tp)
            self._read1_t0[rid] = time.perf_counter()
            self._publish(dst, {"t": "read1", "rid": rid, "src": self.engine_id, "first": first, "last": last})
            self.stats["reads"] += 1
            return
        self._publish_wire({"t": "read", "dst": dst, "rid": req.request_id, "src": self.engine_id,
                            "src_tp": self.tp, "first": first, "last": last})
        self._use_reservation(req.request_id, 1)
        self.dp.post_read(req.request_id, list(req.block_ids[first:last]), dst, src_tp)
        self.stats["reads"] += 1

    def finish_read(self, m) -> None:
        """Every prefill rank (ext event {rid, ok}): unpack the pulled prefix
        and resume the request -- unless it left READING meanwhile (aborted:
        its blocks may belong to another request now), then only drain; or
        unless the decode engine's verdict is false (it no longer held the
        blocks: filler bytes), then drain and let the request recompute."""
        rid, ok = (m, True) if isinstance(m, str) else (m["rid"], bool(m.get("ok", True)))
        sched = self.engine.scheduler
        alive = rid in sched.reading
        if self._read1.pop(rid, None) is not None:  # one-sided: the copy landed, the blocks are the request's again
            sched.release_write(rid)
        if self.dp.finish_read(rid, unpack=alive and ok) and alive:
            self.engine.finish_remote_read(rid, ok)

    def read1_go(self, m: dict) -> None:
        """Every prefill rank (ext event "kv_read1_go", one-sided READ): the
        decode engine pinned (ok) or no longer holds the prefix blocks."""
        rid = m["rid"]
        st = self._read1.get(rid)
        self._read1_t0.pop(rid, None)
        if st is None or rid in self.dp.reads_in:  # (a verdict after the timeout's, or twice)
            return
        sched = self.engine.scheduler
        dst, blocks, src_tp = st
        if m["ok"] and rid in sched.reading:
            try:
                self.dp.read_one_sided(rid, blocks, dst, src_tp, m["blocks"])
                return
            except Exception as e:  # noqa: BLE001 -- mapping the decode cache failed: recompute instead
                log.warning("one-sided READ of %s failed (%s): recomputing the prefix", rid, e)
        # nothing copied: the request recomputes its prefix (or is gone)
        del self._read1[rid]
        sched.release_write(rid)
        if m["ok"]:
            self._publish(dst, {"t": "read1_done", "rid": rid})
        if rid in sched.reading:
            self.engine.finish_remote_read(rid, False)

    def after_step_prefill(self) -> None:
        """Every prefill rank, after each engine step (same step everywhere)."""
        self.dp.end_forward()
        eng = self.engine
        for rid in self._released:
            eng.finish_transfer(rid)
        self._released.clear()
        self.poll_sends()
        self.dp.poll_reads()
        if self.reservations:
            self.gc_reservations()

    def poll_sends(self) -> None:
        """Completed sends recycle their staging; one-sided: a request whose
        writes landed gets its "done" now (or, when its prompt never finished
        in the engine -- aborted mid-forward -- a "fail" telling the decode
        engine the write is over and the request is its own to prefill)."""
        done = self.dp.poll_sends()
        if not self.dp.one_sided:
            return
        self._written.update(done)
        if not self._written:
            return
        reqs = self.engine.requests
        for rid in list(self._written):
            w = self._done_wait.pop(rid, None)
            if w is not None:  # first token sampled and writes landed (in either order: async steps
                self._publish(w[0], w[1])  # sample a step after the forward that wrote the KV)
            elif rid in reqs:
                continue
            elif rid in self._write_dst:  # (not a request's write: e.g. a preflight pattern)
                self._publish(self._write_dst[rid], {"t": "fail", "rid": rid, "written": True})
            self._written.discard(rid)
            self._write_dst.pop(rid, None)

    def pending_sends(self) -> int:
        return len(self.dp.sends)

    # --------------------------------------------------------------- decode side
    def post_recv(self, m: dict) -> None:
        """Every decode rank (ext event "kv_recv"): post the receives of one
        announcement (one prefill engine, its announcement order)."""
        sched = self.engine.scheduler
        bs = self.dp.block_size
        items = []
        for a in m["reqs"]:
            req = sched.remote.get(a["rid"])
            blocks = None
            if req is not None:  # else cancelled meanwhile: the bytes are drained and dropped
                skip = req.num_computed // bs
                blocks = req.block_ids[skip:(len(req.prompt) + bs - 1) // bs]
                assert len(blocks) == a["nblocks"], (len(blocks), a["nblocks"])
            items.append((a["rid"], a["nblocks"], blocks))
        if self.rank == 0:
            for n in m["_bytes"]:
                self.pool.unreserve(n)
        self.dp.post_recv_batch(m["src"], m["src_tp"], items)

    def write_started(self, reqs: list) -> None:
        """Every decode rank (ext event "kv_write_started", one-sided
        transport; [rid, nblocks] pairs): a prefill worker is writing into
        these requests' blocks; an abort now holds the blocks until the write
        is over."""
        sched = self.engine.scheduler
        now = time.perf_counter()
        per_block = self.dp.lay.num_layers * 2 * self.dp.lay.block_bytes
        for rid, nblocks in reqs:
            if rid in sched.remote:
                sched.write_pending.add(rid)
                self._write_t0[rid] = (now, nblocks * per_block)

    def write_aborted(self, rid: str) -> None:
        """Every decode rank (ext event "kv_write_abort", one-sided): the
        prefill worker's write into rid's blocks is over but produced no first
        token; free the blocks of an aborted request, or prefill it here."""
        sched = self.engine.scheduler
        self._write_t0.pop(rid, None)
        if not sched.release_write(rid) and rid in sched.remote:
            self.engine.fallback_local_prefill(rid)

    def read1_pin(self, m: dict) -> None:
        """Every decode rank (ext event "kv_read1_pin", one-sided READ): pin
        the request's prefix blocks [first, last) while a prefill worker
        copies them; the leader names them to it (or says they are gone)."""
        rid = m["rid"]
        blocks = self.read_blocks_of(rid, m["first"], m["last"])
        if blocks is not None:
            self.engine.scheduler.read_pinned.add(rid)
        if self.rank == 0:
            self._publish(m["src"], {"t": "read1_ok", "rid": rid, "ok": blocks is not None, "blocks": blocks or [],
                                     "src": self.engine_id})
        self.stats["served"] += 1
        if blocks is None:
            self.stats["reads_refused"] = self.stats.get("reads_refused", 0) + 1

    def read1_unpin(self, rid: str) -> None:
        """Every decode rank (ext event "kv_read1_unpin"): the copy is over."""
        self.engine.scheduler.unpin_read(rid)

    def write_timed_out(self, rid: str) -> None:
        """Every decode rank (ext event "kv_write_timeout", one-sided): prefill
        the request here; its blocks stay marked as written into, so an abort
        holds them until the writer's "done" / "fail"."""
        sched = self.engine.scheduler
        if rid in sched.remote:
            pending = rid in sched.write_pending
            self.engine.fallback_local_prefill(rid)
            if pending:
                sched.write_pending.add(rid)

    def finish_recv(self, m: dict) -> None:
        """Every decode rank (ext event "kv_finish"): unpack and let the
        request decode (drain only when it was cancelled meanwhile)."""
        rid = m["rid"]
        eng = self.engine
        alive = rid in eng.scheduler.remote
        if self.dp.one_sided:  # the prefill worker wrote the blocks before publishing "done"
            t0, nbytes = self._write_t0.pop(rid, (time.perf_counter(), 0))
            if alive:
                eng.finish_remote_prefill(rid, m["tok"], m["lp"])
                eng.request_timer.observe_transfer(time.perf_counter() - t0, nbytes)
                self.stats["recv"] += 1
            else:
                eng.scheduler.release_write(rid)
            return
        x = self.dp.recvs.get(rid)
        t0, nbytes = (x.t0, x.buf.numel()) if x is not None else (time.perf_counter(), 0)
        with tracing.span("kv_transfer.unpack"):
            done = self.dp.finish_recv(rid, unpack=alive)
        if done and alive:
            eng.finish_remote_prefill(rid, m["tok"], m["lp"])
            eng.request_timer.observe_transfer(time.perf_counter() - t0, nbytes)
            self.stats["recv"] += 1

    def read_blocks_of(self, rid: str, first: int, last: int) -> list[int] | None:
        """The decode engine's blocks [first, last) of a request's prompt, or
        None when it no longer holds them: the request is still waiting for
        its remote prefill, or it fell back to a local prefill (still
        running, blocks allocated and the prefix computed), else gone."""
        sched = self.engine.scheduler
        req = sched.remote.get(rid) or self.engine.requests.get(rid)
        if req is None or len(req.block_ids) < last or req.num_computed < last * self.dp.block_size:
            return None
        return list(req.block_ids[first:last])

    def serve_read(self, m: dict) -> None:
        """Every decode rank (ext event "kv_read"): send this rank's pieces of
        the request's cached blocks [first, last) to the pulling engine, and
        (leader) the verdict whether those were its blocks.  The bytes go
        either way: the prefill rank's receive is posted and wire order needs
        the matching send."""
        n = m["last"] - m["first"]
        blocks = self.read_blocks_of(m["rid"], m["first"], m["last"])
        ok = blocks is not None
        if self.rank == 0:
            self.pool.unreserve(m["_bytes"])
            self._publish(m["src"], {"t": "read_verdict", "rid": m["rid"], "ok": ok})
        self.dp.serve_read(m["rid"], blocks if ok else [0] * n, m["src"], m["src_tp"])
        self.stats["served"] += 1
        if not ok:
            self.stats["reads_refused"] = self.stats.get("reads_refused", 0) + 1

    def after_step_decode(self) -> None:
        self.dp.poll_served()
        self.dp.poll_recvs()

    def take_notifications(self) -> list[dict]:
        out = []
        while self.inbox:
            out.append(self.inbox.popleft())
        return out

    def pending(self) -> int:
        return self.dp.pending() + len(self.inbox)


# ------------------------------------------------------------------ wiring
def install_decode(rep, agent: KVTransferAgent) -> None:
    """Every decode rank: handlers for the leader's ext events."""
    rep.handlers["kv_recv"] = agent.post_recv
    rep.handlers["kv_finish"] = agent.finish_recv
    rep.handlers["kv_read"] = agent.serve_read
    rep.handlers["kv_fallback"] = agent.engine.fallback_local_prefill
    rep.handlers["kv_write_started"] = agent.write_started
    rep.handlers["kv_write_abort"] = agent.write_aborted
    rep.handlers["kv_write_timeout"] = agent.write_timed_out
    rep.handlers["kv_read1_pin"] = agent.read1_pin
    rep.handlers["kv_read1_unpin"] = agent.read1_unpin
    rep.handlers["reset_prefix_cache"] = lambda _: agent.engine.kv.reset_prefix_cache()
    rep.post_step_hooks.append(agent.after_step_decode)


class WireOrder:
    """The decode leader's FIFO of wire messages ("start" announcements and
    "read" requests), in arrival order = the control plane's total order.
    `pop_ready(reserve)` releases messages from the head while their staging
    can be reserved and stops at the first that cannot: a later message never
    overtakes an earlier one, which is what keeps the RCCL wire deadlock-free
    (module docstring).  (Round 5 kept one FIFO per source and per kind, and
    served every source's starts before any read: a decode rank could post a
    WRITE receive ahead of a READ send that the prefill rank had enqueued in
    the opposite order.)"""

    def __init__(self):
        self.q: collections.deque = collections.deque()
        self.deferred = 0

    def push(self, m: dict) -> None:
        self.q.append(m)

    def __len__(self) -> int:
        return len(self.q)

    def pop_ready(self, reserve) -> list[dict]:
        """reserve(m) -> bool: take m's staging (False = not now)."""
        out = []
        while self.q:
            if not reserve(self.q[0]):
                self.deferred += 1
                break
            out.append(self.q.popleft())
        return out


def decode_leader_hook(rep, agent: KVTransferAgent, start_timeout: float | None = None,
                       write_timeout: float | None = None):
    """Engine-thread hook on the decode leader: notifications -> lockstep ext
    events, with staging backpressure (announcements and read requests wait,
    in wire order, until the pool can take their bytes: `WireOrder`).

    Remote prefills whose transfer never starts fall back to a local prefill
    (ext "kv_fallback" on every rank): on a "fail" notification (the prefill
    worker dropped the request before announcing it) or after
    `start_timeout` seconds without an announcement (DX_REMOTE_PREFILL_TIMEOUT_S,
    default 120: the prefill queue is stuck or every prefill worker is gone).
    Safe because no receive was posted for it: a late announcement finds the
    request no longer remote and its bytes are drained (post_recv), a late
    READ gets filler bytes and a false verdict (serve_read), and the fallback
    publishes a wire "cancel" so a prefill worker that has not taken the
    request yet drops it.  Not covered: a prefill worker that dies after
    announcing, mid-WRITE: its receives stay posted until the pair's
    ProcessGroupNCCL watchdog times out (300 s, StoreLinks) and aborts the
    communicator, which fails this worker."""
    wire = WireOrder()
    done: dict[str, dict] = {}
    announced: set[str] = set()
    started: set[str] = set()  # rids whose announcement arrived (receives posted or about to be)
    failed: list[str] = []
    dp, pool = agent.dp, agent.pool
    if start_timeout is None:
        start_timeout = float(os.environ.get("DX_REMOTE_PREFILL_TIMEOUT_S", "120") or 0)
    # one-sided transport: a write announced but not done after this long (the
    # prefill worker died mid-write) -> the request is prefilled here; a writer
    # that is only slow writes the same prompt's KV into the same blocks, and
    # an abort keeps holding the blocks (write_pending stays set)
    if write_timeout is None:
        write_timeout = float(os.environ.get("DX_REMOTE_WRITE_TIMEOUT_S", "120") or 0)
    writing: dict[str, float] = {}
    pinned: dict[str, float] = {}  # one-sided READs in progress: rid -> when the pin was asked
    writer_of: dict[str, str] = {}  # one-sided: rid -> prefill engine that announced the write
    last_writer_scan = [time.perf_counter()]
    sched = agent.engine.scheduler
    last_scan = [time.perf_counter()]

    def fall_back(rid: str) -> None:
        if rid in sched.remote and rid not in started:
            rep.submit("kv_fallback", rid)
            agent._publish_wire({"t": "cancel", "rid": rid})
            agent.stats["fallbacks"] = agent.stats.get("fallbacks", 0) + 1

    def pending() -> int:
        """Notifications not yet turned into events (deferred by backpressure,
        or a "done" whose receives have not landed)."""
        return len(wire) + len(done)

    def reserve(m: dict) -> bool:
        if m["t"] == "start":
            n = [dp.recv_bytes(a["nblocks"], m["src_tp"]) for a in m["reqs"]]
            if not pool.reserve(*n):
                return False
        else:
            n = dp.send_bytes(m["last"] - m["first"], m["src_tp"])
            if not pool.reserve(n):
                return False
        m["_bytes"] = n
        return True

    one_sided = getattr(dp, "one_sided", False)

    def hook():
        for m in agent.take_notifications():
            t = m.get("t", "start")
            if one_sided:  # nothing to post or drain: the prefill worker writes the blocks itself
                if t == "start":
                    rids = [a["rid"] for a in m["reqs"]]
                    started.update(rids)
                    now_w = time.perf_counter()
                    writing.update((r, now_w) for r in rids)
                    writer_of.update((r, m["src"]) for r in rids)
                    rep.submit("kv_write_started", [[a["rid"], a["nblocks"]] for a in m["reqs"]])
                    for rid in rids:
                        agent.span(rid, "start")
                elif t == "done":
                    agent.span(m["rid"], "landed")
                    rep.submit("kv_finish", {"rid": m["rid"], "tok": m["tok"], "lp": m["lp"]})
                    agent.span(m["rid"], "joined")
                elif t == "fail":
                    if m.get("written"):
                        rep.submit("kv_write_abort", m["rid"])
                    else:
                        failed.append(m["rid"])
                elif t == "read1":
                    pinned[m["rid"]] = time.perf_counter()
                    rep.submit("kv_read1_pin", m)
                elif t == "read1_done":
                    pinned.pop(m["rid"], None)
                    rep.submit("kv_read1_unpin", m["rid"])
                continue
            if t == "start":
                wire.push(m)
                started.update(a["rid"] for a in m["reqs"])
                for a in m["reqs"]:
                    agent.span(a["rid"], "start")
            elif t == "read":
                wire.push(m)
            elif t == "done":
                done[m["rid"]] = m
                agent.span(m["rid"], "done")
            elif t == "fail":
                failed.append(m["rid"])
        while failed:
            fall_back(failed.pop())
        now = time.perf_counter()
        if (start_timeout or write_timeout) and now - last_scan[0] > 0.5:
            last_scan[0] = now
            for rid, r in list(sched.remote.items()):
                if start_timeout and rid not in started and r.admit_time and now - r.admit_time > start_timeout:
                    log.warning("remote prefill of %s did not start in %.0fs: prefilling locally", rid,
                                start_timeout)
                    fall_back(rid)
            for rid, t0 in list(pinned.items()):  # a reader that died mid-copy never says "read1_done"
                if write_timeout and now - t0 > write_timeout:
                    log.warning("one-sided READ of %s not done in %.0fs: unpinning", rid, write_timeout)
                    del pinned[rid]
                    rep.submit("kv_read1_unpin", rid)
            for rid, t0 in list(writing.items()):
                if rid not in sched.remote:
                    del writing[rid]
                elif write_timeout and now - t0 > write_timeout:
                    log.warning("one-sided write of %s not done in %.0fs: prefilling locally", rid, write_timeout)
                    del writing[rid]
                    rep.submit("kv_write_timeout", rid)
                    agent.stats["write_timeouts"] = agent.stats.get("write_timeouts", 0) + 1
        if writer_of and now - last_writer_scan[0] > min(10.0, write_timeout or 10.0):
            # a prefill worker whose lease is gone will never say "done" / "fail":
            # its writes are over -- release their blocks (prefill here what still waits)
            last_writer_scan[0] = now
            pending_w = sched.write_pending
            # (a rid still REMOTE_PREFILLING may not have had its kv_write_started
            # applied yet: keep it until it is neither waiting nor written into)
            for rid in [r for r in writer_of if r not in pending_w and r not in sched.remote]:
                del writer_of[rid]
            gone: dict[str, bool] = {}
            for rid, src in list(writer_of.items()):
                if src not in gone:
                    gone[src] = agent.engine_gone(src)
                if gone[src]:
                    log.warning("prefill engine %s is gone: releasing the write into %s", src, rid)
                    del writer_of[rid]
                    writing.pop(rid, None)
                    rep.submit("kv_write_abort", rid)
        if len(started) > 4096:  # finished rids no longer pending
            started.intersection_update(set(sched.remote) | set(dp.recvs))
        before = wire.deferred
        for m in wire.pop_ready(reserve):
            if m["t"] == "start":
                rep.submit("kv_recv", m)
                for a in m["reqs"]:
                    agent.span(a["rid"], "posted")
            else:
                rep.submit("kv_read", m)
        agent.stats["deferred"] += wire.deferred - before
        for rid in dp.recvs_landed():
            agent.span(rid, "landed")
            m = done.get(rid)
            if m is not None and rid not in announced:
                announced.add(rid)
                del done[rid]
                rep.submit("kv_finish", {"rid": rid, "tok": m["tok"], "lp": m["lp"]})
                agent.span(rid, "joined")
        if len(announced) > 4096:  # finished rids no longer pending
            announced.intersection_update(dp.recvs.keys())

    hook.pending = pending
    return hook


def install_prefill(rep, agent: KVTransferAgent) -> None:
    """Every prefill rank: announce + stream on the layer hook, release the
    blocks on the first token (same step on every rank), unpack pulled
    prefixes on the leader's event."""
    eng = rep.engine
    agent._released = []
    eng.batch_hook = agent.on_batch
    eng.model.layer_hook = agent.dp.on_layer
    eng.prefill_done_hook = agent.on_prefilled
    eng.scheduler.on_remote_read = agent.on_read
    rep.handlers["kv_read_done"] = agent.finish_read
    rep.handlers["kv_read1_go"] = agent.read1_go
    rep.post_step_hooks.append(agent.after_step_prefill)


def prefill_leader_hook(rep, agent: KVTransferAgent):
    """Engine-thread hook on the prefill leader (every engine-loop iteration,
    idle or not): completed sends recycle their staging; landed prefix pulls
    become lockstep "kv_read_done" events."""
    announced: set[str] = set()
    verdicts = agent.read_verdicts
    eng = agent.engine
    seen_cancel = [0]
    last_gc = [time.perf_counter()]
    read_timeout = float(os.environ.get("DX_REMOTE_READ_TIMEOUT_S", "30") or 30)

    def hook():
        if agent._ipc_by_key and time.perf_counter() - last_gc[0] > 10.0:  # departed decode engines' caches
            last_gc[0] = time.perf_counter()
            agent.gc_peers()
        if agent._read1_t0:  # one-sided READs the decode engine never answered: recompute the prefix
            now = time.perf_counter()
            for rid, t0 in list(agent._read1_t0.items()):
                if now - t0 > read_timeout:
                    log.warning("one-sided READ of %s unanswered for %.0fs: recomputing the prefix", rid, read_timeout)
                    del agent._read1_t0[rid]
                    rep.submit("kv_read1_go", {"rid": rid, "ok": False, "blocks": []})
        # sends complete asynchronously: poll them here too, not only after
        # engine steps, or the last transfer before an idle period keeps its
        # staging (and a draining worker waits on it forever)
        agent.poll_sends()
        for m in agent.take_notifications():
            if m.get("t") == "read_verdict":
                verdicts[m["rid"]] = bool(m["ok"])
            elif m.get("t") == "read1_ok":  # one-sided READ: copy (or give up) on every rank
                if m["rid"] not in agent._read1:  # answered after the READ timed out: unpin at once
                    if m["ok"]:
                        agent._publish(m["src"], {"t": "read1_done", "rid": m["rid"]})
                    continue
                if m["ok"]:
                    verdicts[m["rid"]] = True
                rep.submit("kv_read1_go", m)
        if agent.cancel_seq != seen_cancel[0]:  # decode engines gave these up: drop the ones not started
            seen_cancel[0] = agent.cancel_seq
            for r in list(eng.scheduler.waiting):
                if r.request_id in agent.cancelled and r.remote_decode:
                    rep.abort(r.request_id)
        if agent.reservations:  # also while steps fail: dropped requests notify their decode engine
            agent.gc_reservations()
        for rid in agent.dp.reads_landed():
            if rid not in announced and rid in verdicts:  # bytes landed and the decode engine said what they are
                announced.add(rid)
                rep.submit("kv_read_done", {"rid": rid, "ok": verdicts.pop(rid)})
                st = agent._read1.get(rid)
                if st is not None:  # one-sided: the decode engine may unpin its blocks now
                    agent._publish(st[0], {"t": "read1_done", "rid": rid})
        if len(announced) > 4096:
            announced.intersection_update(agent.dp.reads_in.keys())

    return hook


def follower_setup(rep, role: str, cp_address: str, engine_id: str, namespace: str, lease_id: int | None,
                   kv_transport: str | None = None) -> None:
    """Runs on TP follower ranks (spawned processes): own control-plane client,
    own transfer endpoint, handlers for the leader's events."""
    from ..runtime.control_plane import SyncControlPlaneClient

    sc = SyncControlPlaneClient(cp_address)
    agent = KVTransferAgent(rep.engine, _CP(sc.client, sc.loop), engine_id, namespace, rep.rank, rep.world,
                            kv_transport=kv_transport)
    agent.start_sync(lease_id)
    rep._kv_agent, rep._cp_client = agent, sc
    if role == "decode":
        install_decode(rep, agent)
    else:
        install_prefill(rep, agent)
