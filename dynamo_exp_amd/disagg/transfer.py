"""Prefill -> decode KV block transfer over RCCL (xGMI): the NIXL data plane.

ONE data plane (`KVDataPlane`) serves both the `dynamo serve` disaggregated
graphs (disagg/agent.py wires it to independently started workers) and the
headline benchmark (disagg/bench_disagg.py); only how a rank reaches its
peer differs (`WorldLinks`: ranks of one torch.distributed world;
`StoreLinks` in agent.py: per-pair process groups built on the decode rank's
TCPStore).  Reference behaviour:

* WRITE, layer-streamed (reference CopyStream / trigger_layer,
  lib/llm/src/kv/layer.rs:785-1130; NIXL write_blocks, Patch:1361-1424): the
  prefill ranks announce a request before the forward pass that completes its
  prompt; at the end of each layer group the group's KV is packed on a copy
  stream (which waits only for that layer's event, so later layers keep
  computing) and sent, one message per (layer group, relayout piece).  The
  decode ranks post the receives when the announcement arrives, unpack into
  the request's pre-allocated blocks when the sender's first token arrived
  and their receives landed, and the request joins the decode batch.
* READ (reference Patch:1296-1360 read_blocks): a prefill engine that lacks a
  prompt prefix the decode engine caches pulls those blocks over the
  reverse-direction links instead of recomputing them.
* TP relayout (reference block_copy.cu:558-758 permute_scatter, Triton
  kv_rearrange Patch:908-1039): the cache block is [Hkv_local][BS][D], so a
  rank's KV heads are one contiguous byte range of every block;
  `tp_relayout_plan` turns (prefill TP, decode TP) into (src rank, dst rank,
  src offset, dst offset, length) pieces that the pack/unpack kernel
  (csrc/kernels/kv_copy.hip) applies to all blocks and layers of a group in
  one launch.  Each rank sends / receives only its own pieces.
* One-sided WRITE (`one_sided=True`, the `ipc` transport; round 6): the
  prefill rank writes each layer group's relayout pieces STRAIGHT into the
  decode rank's KV blocks through its mapping of the decode cache (kv_share.py)
  (`remote_kv(engine, rank)` -> pointer + layout), one block-copy launch per
  (group, piece) on the copy stream -- no staging, no receive kernel, nothing
  that waits on a peer: the NIXL WRITE of the reference (Patch:1361-1424)
  with the GPU's own memory fabric (xGMI between GPUs, the device's HBM
  between two processes on one GPU).  Completion is the copy stream's event;
  the agent publishes the request's "done" only after it.
* Staging is pooled with backpressure: a buffer is only handed out against
  a reservation (`StagingPool.reserve`) or when the pool is under its cap;
  prefill engines admit work, and decode engines post receives / serve
  reads, only while their pool can take the bytes.

Ordering: RCCL matches a pair's point-to-point messages strictly in order,
so both sides post them in the same order: layer-group major, then the
announcement's request order, then plan piece order.  Opposite directions
use separate links (their own communicators), so an in-order RCCL stream
never interleaves a pair's sends and receives.

Lockstep (TP > 1): every rank of an engine runs the same schedule
(parallel/tp.py), so `begin_send`, `on_layer`, `end_forward`,
`post_recv_batch`, `finish_recv`, `serve_read`, `post_read` and
`finish_read` are called in the same order on every rank; only "did my
receive land" is rank-local and is turned into a lockstep event by the
engine leader.  Block ownership changes (freeing a prefill request's blocks,
finishing a decode request's remote prefill) therefore happen at the same
step on every rank: a prefill request's blocks are released right after its
first token, because `end_forward` orders the compute stream after every
pack of the forward (the bytes live in staging from then on).
"""
from __future__ import annotations

import collections
import logging
import threading
import time
from dataclasses import dataclass, field

import torch

from .. import ops
from ..utils import streams
from ..utils.faults import FAULTS

log = logging.getLogger("dynamo_exp_amd.disagg")


@dataclass
class KVLayout:
    num_layers: int
    num_blocks: int
    block_bytes: int  # one (layer, K|V) block: Hkv * BS * D * elem

    @classmethod
    def of(cls, kv_cache: torch.Tensor) -> "KVLayout":
        L, two, NB, H, BS, D = kv_cache.shape
        return cls(L, NB, H * BS * D * kv_cache.element_size())

    @property
    def prefix(self) -> int:
        return self.num_layers * 2

    @property
    def prefix_stride(self) -> int:
        return self.num_blocks * self.block_bytes


@dataclass
class RemoteKV:
    """A peer rank's KV cache as the one-sided transport sees it: a device
    pointer (mapped from its shared chunks) or, for in-process engines, the tensor itself, and
    its layout (the cache is [L, 2, num_blocks, Hkv, BS, D])."""

    num_blocks: int
    block_bytes: int
    num_layers: int
    ptr: int | None = None
    tensor: torch.Tensor | None = None


@dataclass
class RelayoutPiece:
    src_rank: int  # prefill TP rank
    dst_rank: int  # decode TP rank
    src_inner_off: int  # bytes into the prefill rank's (layer, K|V) block
    dst_inner_off: int  # bytes into the decode rank's block
    nbytes: int  # contiguous bytes per (layer, K|V, block)


def kv_heads_of_rank(rank: int, tp: int, total_kv_heads: int) -> tuple[int, int]:
    """(first KV head, count) held by a TP rank: a contiguous slice when the
    heads divide over the ranks, else one replicated head per rank
    (models/llama.py: n_kv = 1 when num_key_value_heads < tp)."""
    if total_kv_heads >= tp:
        n = total_kv_heads // tp
        return rank * n, n
    return (rank * total_kv_heads) // tp, 1


def tp_relayout_plan(prefill_tp: int, decode_tp: int, total_kv_heads: int, block_size: int, head_dim: int,
                     elem: int = 2) -> list[RelayoutPiece]:
    """Which head sub-range of each prefill rank's blocks lands where on which
    decode rank.  Each decode rank takes every head it holds from the first
    prefill rank holding it (replicated heads when a TP size exceeds the KV
    head count); pieces are in ascending head order, the order both sides
    post their sends / receives in."""
    for tp in (prefill_tp, decode_tp):
        if total_kv_heads >= tp and total_kv_heads % tp:
            raise ValueError("KV heads must divide the TP size (or be fewer than it)")
        if total_kv_heads < tp and tp % total_kv_heads:
            raise ValueError("TP size must be a multiple of the KV head count when it exceeds it")
    head_bytes = block_size * head_dim * elem
    pieces: list[RelayoutPiece] = []
    for d in range(decode_tp):
        dh0, dn = kv_heads_of_rank(d, decode_tp, total_kv_heads)
        for h in range(dh0, dh0 + dn):
            for p in range(prefill_tp):
                ph0, pn = kv_heads_of_rank(p, prefill_tp, total_kv_heads)
                if ph0 <= h < ph0 + pn:
                    break
            so, do = (h - ph0) * head_bytes, (h - dh0) * head_bytes
            last = pieces[-1] if pieces else None
            if (last is not None and last.src_rank == p and last.dst_rank == d
                    and last.src_inner_off + last.nbytes == so and last.dst_inner_off + last.nbytes == do):
                last.nbytes += head_bytes
            else:
                pieces.append(RelayoutPiece(p, d, so, do, head_bytes))
    return pieces


def block_ids_tensor(block_ids, device) -> torch.Tensor:
    """int32 block ids on `device` WITHOUT a host synchronisation: on a GPU
    the list goes through pinned memory with a non-blocking H2D on the
    current stream (PyTorch's pinned allocator keeps the host block until
    that copy ran), so the copy orders with the kernels that consume it.  A
    pageable `torch.tensor(..., device=cuda)` would block the host until the
    current stream drained -- inside the prefill forward's layer hooks that
    stalls the host at every layer group."""
    if isinstance(block_ids, torch.Tensor):
        return block_ids
    t = torch.tensor(block_ids, dtype=torch.int32)
    dev = torch.device(device)
    if dev.type != "cuda":
        return t
    return t.pin_memory().to(dev, non_blocking=True)


_ARANGE: dict = {}


def _arange(n: int, device) -> torch.Tensor:
    """Cached device [0, n) (a kernel launch once per size, never a sync)."""
    dev = torch.device(device)
    lst = _ARANGE.setdefault(dev, [])
    if not lst or lst[-1].numel() < n:  # outgrown ones stay alive: other streams may still read them
        lst.append(torch.arange(max(n, 16384), dtype=torch.int32, device=dev))
    return lst[-1][:n]


def pack_blocks(kv_cache: torch.Tensor, block_ids, inner_off: int = 0, inner_bytes: int | None = None,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """Gather blocks (all layers, K and V) into [L*2, n, inner] bytes.
    `block_ids`: list, or an int32 tensor on the cache's device
    (`block_ids_tensor`) built once per transfer."""
    lay = KVLayout.of(kv_cache)
    n = len(block_ids)
    inner = inner_bytes or lay.block_bytes
    if out is None:
        out = torch.empty(lay.prefix * n * inner, dtype=torch.uint8, device=kv_cache.device)
    dev = kv_cache.device
    ops.kv_copy_blocks(out, kv_cache, block_ids_tensor(block_ids, dev), _arange(n, dev), lay.prefix,
                       lay.prefix_stride, n * inner, lay.block_bytes, inner, inner, src_inner_off=inner_off)
    return out


def unpack_blocks(kv_cache: torch.Tensor, staging: torch.Tensor, block_ids, inner_off: int = 0,
                  inner_bytes: int | None = None) -> None:
    lay = KVLayout.of(kv_cache)
    n = len(block_ids)
    inner = inner_bytes or lay.block_bytes
    dev = kv_cache.device
    ops.kv_copy_blocks(kv_cache, staging, _arange(n, dev), block_ids_tensor(block_ids, dev), lay.prefix,
                       n * inner, lay.prefix_stride, inner, lay.block_bytes, inner, dst_inner_off=inner_off)


def transfer_bytes(kv_cache: torch.Tensor, n_blocks: int) -> int:
    lay = KVLayout.of(kv_cache)
    return lay.prefix * n_blocks * lay.block_bytes


class StagingPool:
    """Reusable staging buffers for KV transfers (device memory, or pinned host
    memory for host-staged transport), in size classes of `granule` bytes, so
    a 3000-token Llama-3-8B request does not allocate ~375 MiB per transfer on
    each side.

    Backpressure: `cap` bounds the bytes handed out plus the bytes promised
    to admitted work (`reserve`).  A caller that admits work (a prefill
    engine pulling the queue, a decode engine posting receives) asks
    `can_take` / `reserve` first and defers when the answer is no; `take`
    itself never refuses (TP followers take what their leader admitted), but
    counts any overshoot in `stats["over_cap"]`.  A single transfer larger
    than the cap is admitted when the pool is idle, so progress is
    guaranteed.  A buffer goes back with `give` once every stream that used
    it is done with it."""

    def __init__(self, device, cap_bytes: int = 4 << 30, granule: int = 8 << 20, pinned: bool = False):
        self.device = torch.device(device)
        self.cap = cap_bytes
        self.granule = granule
        self.pinned = pinned
        self.free: dict[int, list[torch.Tensor]] = collections.defaultdict(list)
        self.in_use = 0
        self.reserved = 0  # bytes promised to admitted, not yet started transfers
        self.held = 0  # bytes owned by the pool (free + in use)
        self.stats = dict(allocs=0, reuses=0, over_cap=0, deferred=0, peak=0)
        # admission (a worker's event loop) and transfers (the engine thread)
        # touch the counters from different threads
        self._lock = threading.Lock()

    def _cls(self, nbytes: int) -> int:
        return max(self.granule, -(-nbytes // self.granule) * self.granule)

    def can_take(self, nbytes: int) -> bool:
        idle = self.in_use == 0 and self.reserved == 0
        return idle or self.in_use + self.reserved + self._cls(nbytes) <= self.cap

    def reserve(self, *nbytes: int) -> bool:
        """Promise buffers of these sizes to work being admitted (all or
        none); False = defer it.  Each is released with `unreserve(n)`."""
        c = sum(self._cls(n) for n in nbytes if n)
        with self._lock:
            idle = self.in_use == 0 and self.reserved == 0
            if not (idle or self.in_use + self.reserved + c <= self.cap):
                self.stats["deferred"] += 1
                return False
            self.reserved += c
            return True

    def unreserve(self, nbytes: int) -> None:
        if nbytes:
            with self._lock:
                self.reserved = max(0, self.reserved - self._cls(nbytes))

    def take(self, nbytes: int) -> torch.Tensor:
        c = self._cls(nbytes)
        with self._lock:
            if self.in_use + self.reserved + c > self.cap and self.in_use > 0:
                self.stats["over_cap"] += 1
            lst = self.free.get(c)
            buf = lst.pop() if lst else None
            self.in_use += c
            self.stats["peak"] = max(self.stats["peak"], self.in_use)
        if buf is not None:
            self.stats["reuses"] += 1
        else:
            # a normal tensor even when first taken inside inference mode (the
            # preflight, a forward's layer hook): pooled buffers are written
            # later by handlers that run outside it, and an inference tensor
            # refuses in-place updates there (found by the 70B@20 rehearsal)
            with torch.inference_mode(False):
                if self.pinned:
                    buf = torch.empty(c, dtype=torch.uint8).pin_memory()
                else:
                    buf = torch.empty(c, dtype=torch.uint8, device=self.device)
            with self._lock:
                self.held += c
            self.stats["allocs"] += 1
        return buf

    def give(self, buf: torch.Tensor) -> None:
        c = buf.numel()
        with self._lock:
            self.in_use -= c
            if self.held - self.in_use > self.cap:  # over the cap: let it go
                self.held -= c
                return
            self.free[c].append(buf)


def layer_groups(num_layers: int, groups: int) -> list[tuple[int, int]]:
    """[l0, l1) ranges of the layer groups a request's KV streams in."""
    groups = max(1, min(groups, num_layers))
    step = -(-num_layers // groups)
    return [(l0, min(num_layers, l0 + step)) for l0 in range(0, num_layers, step)]


# ---------------------------------------------------------------------------- links
class WorldLinks:
    """Peers that are ranks of this process's torch.distributed world (the
    benchmark: every prefill and decode rank of the node in one world).
    `ranks_of[engine_id]` lists the global ranks of an engine's TP ranks.
    WRITE traffic uses `group`, READ traffic `rev_group` (its own RCCL
    communicators, so the two directions never share an in-order stream).
    RCCL point-to-point builds one communicator per rank pair on first use;
    `warm` creates them all up front (collectively), since creating one
    lazily inside the serving loop blocks until the peer also reaches it."""

    def __init__(self, ranks_of: dict[str, list[int]], group=None, rev_group=None):
        self.ranks_of = ranks_of
        self.group, self.rev_group = group, rev_group if rev_group is not None else group

    def _dst(self, engine: str, rank: int) -> int:
        return self.ranks_of[engine][rank]

    def send(self, engine: str, rank: int, t: torch.Tensor, rev: bool = False):
        import torch.distributed as dist

        return dist.isend(t, self._dst(engine, rank), group=self.rev_group if rev else self.group)

    def recv(self, engine: str, rank: int, t: torch.Tensor, rev: bool = False):
        import torch.distributed as dist

        return dist.irecv(t, self._dst(engine, rank), group=self.rev_group if rev else self.group)

    def warm(self, me: int, prefill_engines: list[str], decode_engines: list[str], device) -> None:
        """Collective over the world: one message on every (prefill rank,
        decode rank) pair in each direction, in one global order."""
        import torch.distributed as dist

        t = torch.zeros(1, device=device)
        for pe in prefill_engines:
            for p in self.ranks_of[pe]:
                for de in decode_engines:
                    for d in self.ranks_of[de]:
                        if me == p:
                            dist.send(t, d, group=self.group)
                            dist.recv(t, d, group=self.rev_group)
                        elif me == d:
                            dist.recv(t, p, group=self.group)
                            dist.send(t, p, group=self.rev_group)
        if torch.device(device).type == "cuda":
            torch.cuda.synchronize(device)


class _LoopWork:
    """An in-process point-to-point work with the RCCL work contract the data
    plane relies on: `is_completed()` polls without blocking (an event query
    on GPUs), `wait()` orders the *current stream* after the transfer (a
    device-side event wait, never a host block).  A work is matched when its
    peer posts; `wait()` is only legal after `is_completed()`."""

    __slots__ = ("event", "flag", "error")

    def __init__(self):
        self.event = None  # GPU: completion event of the device copy
        self.flag = threading.Event()  # matched (and, on CPU, copied)
        self.error = None

    def is_completed(self) -> bool:
        if not self.flag.is_set():
            return False
        return self.event is None or self.event.query()

    def wait(self) -> None:
        if self.event is None:  # CPU: block until the peer posted (helper threads only)
            self.flag.wait()
            if self.error is not None:
                raise self.error
            return
        torch.cuda.current_stream().wait_event(self.event)


class LoopbackHub:
    """The shared 'wire' of LoopbackLinks: a prefill engine and a decode engine
    in ONE process (on one GPU) exchange KV through the exact data-plane code
    path of the multi-GPU deployment -- same pack/unpack kernels, copy
    streams, events and posting order -- with each matched (send, recv) pair
    executed as one device-to-device copy on the hub's own stream, which
    waits only for the events both sides recorded when they posted.  Messages
    of one (src, dst, direction) channel match strictly in order, like RCCL
    point-to-point.  Used by the one-GPU 1P1D test of the device path
    (tests/test_disagg_gpu.py) and by `tools/loopback_disagg.py`."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.gpu else None
        self.chans: dict[tuple, tuple] = {}
        self._lock = threading.Lock()
        self.stats = dict(copies=0, bytes=0)

    def post(self, chan: tuple, side: int, t: torch.Tensor) -> _LoopWork:
        w = _LoopWork()
        ev = None
        if self.gpu:  # the poster's stream has enqueued everything that fills / frees t
            ev = torch.cuda.Event()
            ev.record()
        with self._lock:
            q = self.chans.get(chan)
            if q is None:
                q = self.chans[chan] = (collections.deque(), collections.deque())
            q[side].append((t, ev, w))
            pairs = []
            while q[0] and q[1]:
                pairs.append((q[0].popleft(), q[1].popleft()))
        for s, r in pairs:
            self._copy(chan, s, r)
        return w

    def _copy(self, chan, s, r) -> None:
        (src, sev, sw), (dst, rev, rw) = s, r
        if src.numel() != dst.numel() or src.dtype != dst.dtype:
            err = RuntimeError(f"loopback {chan}: send of {src.numel()} x {src.dtype} matched a receive of "
                               f"{dst.numel()} x {dst.dtype} (posting order differs between the sides)")
            for w in (sw, rw):
                w.error = err
                w.flag.set()
            raise err
        if self.gpu:
            self.stream.wait_event(sev)
            self.stream.wait_event(rev)
            with torch.cuda.stream(self.stream):
                dst.copy_(src, non_blocking=True)
                done = torch.cuda.Event()
                done.record(self.stream)
            sw.event = rw.event = done
        else:
            dst.copy_(src)
        self.stats["copies"] += 1
        self.stats["bytes"] += dst.numel() * dst.element_size()
        sw.flag.set()
        rw.flag.set()


class LoopbackLinks:
    """Links of one engine rank (`engine`, `rank`) on a LoopbackHub: the same
    `send` / `recv` signature as WorldLinks / StoreLinks.  A channel is
    (src engine, src rank, dst engine, dst rank, reverse?)."""

    def __init__(self, hub: LoopbackHub, engine: str, rank: int = 0):
        self.hub, self.engine, self.rank = hub, engine, rank

    def send(self, engine: str, rank: int, t: torch.Tensor, rev: bool = False):
        return self.hub.post((self.engine, self.rank, engine, rank, rev), 0, t)

    def recv(self, engine: str, rank: int, t: torch.Tensor, rev: bool = False):
        return self.hub.post((engine, rank, self.engine, self.rank, rev), 1, t)


# ---------------------------------------------------------------------------- data plane
@dataclass
class _Seg:
    gi: int  # layer group
    piece: RelayoutPiece
    off: int  # byte offset in the request's staging buffer
    nbytes: int


@dataclass
class _Xfer:
    """One request's KV on this rank (either direction)."""

    rid: str
    peer: str  # peer engine id
    block_ids: list[int] | None  # None: the local request is gone, drain only
    segs: list[_Seg]
    buf: torch.Tensor | None
    ids: torch.Tensor | None = None  # block_ids on the device (built once, on the copy stream)
    works: list = field(default_factory=list)  # [work, done]
    packed: int = 0  # layer groups packed + posted (sender)
    t0: float = 0.0
    event: object = None  # unpack completion (receiver)
    meta: dict = field(default_factory=dict)


class KVDataPlane:
    """One rank's end of the P->D KV data plane.  See the module docstring.

    `links` reaches a peer engine's TP rank; `tp_rank` / `tp_size` place this
    rank in its engine; `total_kv_heads` is the model's KV head count (the
    relayout plan's domain).  Prefill side: `begin_send` (before the forward),
    `on_layer` (model layer hook), `end_forward`, `poll_sends`; READ:
    `post_read`, `reads_landed`, `finish_read`.  Decode side:
    `post_recv_batch`, `recvs_landed`, `finish_recv`; READ: `serve_read`,
    `poll_served`."""

    def __init__(self, kv_cache: torch.Tensor, links, tp_rank: int = 0, tp_size: int = 1,
                 total_kv_heads: int | None = None, host_staging: bool = False, layer_group_count: int = 4,
                 pool_cap_bytes: int = 4 << 30, one_sided: bool = False, remote_kv=None):
        self.kv = kv_cache
        self.links = links
        # one-sided WRITE (module docstring): remote_kv(engine, rank) -> RemoteKV
        self.one_sided = one_sided
        self.remote_kv = remote_kv
        if one_sided and remote_kv is None:
            raise ValueError("one-sided transport needs a remote_kv resolver")
        self.rank, self.tp = tp_rank, tp_size
        L, _, NB, Hl, BS, D = kv_cache.shape
        self.block_size, self.head_dim = BS, D
        self.total_kv_heads = total_kv_heads or Hl * tp_size
        # host_staging: payloads cross through pinned host memory over gloo
        # links (single-GPU functional tests of the disagg path; not the fast path)
        self.host_staging = host_staging
        self.gpu = kv_cache.is_cuda
        self.lay = KVLayout.of(kv_cache)
        self.groups = layer_groups(self.lay.num_layers, layer_group_count)
        # high priority (utils/streams.py): an unpack the decode step waits on
        # never queues behind a spinning RCCL receive
        self.copy_stream = streams.stream("kv_copy", kv_cache.device) if self.gpu else None
        self.pool = StagingPool("cpu" if (host_staging or not self.gpu) else kv_cache.device, pool_cap_bytes,
                                pinned=host_staging and self.gpu)
        self.sends: dict[str, _Xfer] = {}
        self.recvs: dict[str, _Xfer] = {}
        self.reads_in: dict[str, _Xfer] = {}  # prefill side: prefix blocks being pulled
        self.served: collections.deque = collections.deque()  # decode side: served reads in flight
        self._streaming: list[_Xfer] = []  # sends announced for the current forward
        self._plans: dict[tuple, list] = {}
        self.stats = dict(sent_bytes=0, recv_bytes=0, sends=0, recvs=0, send_time=0.0, recv_time=0.0,
                          read_bytes=0, reads=0, served=0, dropped=0)
        # gloo p2p work never reports completion by polling (is_completed stays
        # False) and a wait() with a timeout tears the pair down, so gloo works
        # are waited on by a helper thread each and polled through its flag:
        # the serving loop never blocks on a peer that has not posted yet
        self.blocking = (not self.gpu) or host_staging

    # ------------------------------------------------------------ layout
    def plan(self, prefill_tp: int, decode_tp: int) -> list[RelayoutPiece]:
        key = (prefill_tp, decode_tp)
        p = self._plans.get(key)
        if p is None:
            p = self._plans[key] = tp_relayout_plan(prefill_tp, decode_tp, self.total_kv_heads, self.block_size,
                                                    self.head_dim, self.kv.element_size())
        return p

    def _segs(self, pieces: list[RelayoutPiece], nblocks: int, groups=None) -> list[_Seg]:
        """Segments of one request in posting order: layer group major, then
        plan piece order; contiguous offsets in its staging buffer."""
        out, off = [], 0
        for gi, (l0, l1) in enumerate(self.groups if groups is None else groups):
            for pc in pieces:
                n = (l1 - l0) * 2 * nblocks * pc.nbytes
                out.append(_Seg(gi, pc, off, n))
                off += n
        return out

    def send_bytes(self, nblocks: int, dst_tp: int) -> int:
        """Staging bytes this rank needs to WRITE nblocks to a TP-dst_tp engine."""
        return sum(s.nbytes for s in self._segs(self._my(self.tp, dst_tp, "src"), nblocks))

    def recv_bytes(self, nblocks: int, src_tp: int) -> int:
        return sum(s.nbytes for s in self._segs(self._my(src_tp, self.tp, "dst"), nblocks))

    def _my(self, prefill_tp: int, decode_tp: int, side: str) -> list[RelayoutPiece]:
        plan = self.plan(prefill_tp, decode_tp)
        return [p for p in plan if (p.src_rank if side == "src" else p.dst_rank) == self.rank]

    def _ctx(self):
        return torch.cuda.stream(self.copy_stream) if self.copy_stream is not None else _nullctx()

    def _ids(self, block_ids) -> torch.Tensor | None:
        """A transfer's block ids as a device tensor, enqueued once on the
        copy stream (pinned, non-blocking: no host sync), ahead of the packs /
        unpacks that read them on that same stream."""
        if block_ids is None:
            return None
        with self._ctx():
            return block_ids_tensor(block_ids, self.kv.device)

    def _track(self, work) -> list:
        """[work, done(, waiter thread)] for a posted send / receive."""
        w = [work, False]
        if self.blocking:
            def wait(w=w):
                try:
                    work.wait()
                except Exception as e:  # noqa: BLE001 -- surfaced by _done
                    w.append(e)
                w[1] = True
            t = threading.Thread(target=wait, daemon=True, name="dx-kv-wait")
            t.start()
        return w

    def _done(self, w: list) -> bool:
        if not w[1] and not self.blocking:
            w[1] = w[0].is_completed()
        if w[1] and len(w) > 2:
            raise RuntimeError(f"KV transfer failed: {w[2]!r}")
        return w[1]

    def _wait(self, w: list) -> None:
        """Order the current stream after a work (RCCL: device-side wait, the
        host does not block); gloo: the work already completed (callers
        only finish landed transfers)."""
        if self.blocking:
            while not self._done(w):
                time.sleep(0.0002)
        else:
            w[0].wait()

    def _pack_seg(self, x: _Xfer, seg: _Seg) -> torch.Tensor:
        """Pack one segment (layer group x piece) of x's blocks on the current
        stream; returns the wire view."""
        l0, l1 = self.groups[seg.gi]
        view = x.buf[seg.off:seg.off + seg.nbytes]
        pc = seg.piece
        if self.host_staging:  # pack on the device, then through pinned host memory
            tmp = pack_blocks(self.kv[l0:l1], x.ids, inner_off=pc.src_inner_off, inner_bytes=pc.nbytes)
            view.copy_(tmp)
            torch.cuda.current_stream().synchronize()
        else:
            pack_blocks(self.kv[l0:l1], x.ids, inner_off=pc.src_inner_off, inner_bytes=pc.nbytes, out=view)
        return view

    def _unpack(self, x: _Xfer, unpack: bool) -> None:
        """Copy stream: wait for x's receives (GPU-side), unpack its segments
        into its blocks (unless the request is gone), order the compute stream
        after the unpack; staging retires when the copy stream passed it."""
        with self._ctx():
            for w in x.works:
                self._wait(w)  # the copy stream waits for the RCCL stream (no host block)
            if unpack and x.block_ids is not None:
                for seg in x.segs:
                    l0, l1 = self.groups[seg.gi]
                    src = x.buf[seg.off:seg.off + seg.nbytes]
                    FAULTS.corrupt_received(src)
                    if self.host_staging:
                        src = src.to(self.kv.device, non_blocking=True)
                    unpack_blocks(self.kv[l0:l1], src, x.ids, inner_off=seg.piece.dst_inner_off,
                                  inner_bytes=seg.piece.nbytes)
        if self.copy_stream is not None:
            x.event = torch.cuda.Event()
            x.event.record(self.copy_stream)
            if unpack:
                torch.cuda.current_stream(self.kv.device).wait_event(x.event)  # readers of the blocks wait
        else:
            x.event = True

    def _retire(self, table: dict, timer: str | None) -> None:
        for rid, x in list(table.items()):
            if x.event is None:
                continue
            if x.event is True or x.event.query():
                del table[rid]
                if x.buf is not None:  # (one-sided transfers take no staging)
                    self.pool.give(x.buf)
                if timer:
                    self.stats[timer] += time.perf_counter() - x.t0

    # ------------------------------------------------------------ prefill side: WRITE
    def begin_send(self, rid: str, block_ids: list[int], dst_engine: str, dst_tp: int = 1,
                   dst_block_ids: list[int] | None = None) -> dict:
        """Announce a request whose prompt completes in the coming forward
        (every rank of the prefill engine, same order); returns the
        announcement entry the decode engine needs to post its receives.
        One-sided: `dst_block_ids` are the decode engine's blocks the pieces
        are written into (same length as block_ids)."""
        segs = self._segs(self._my(self.tp, dst_tp, "src"), len(block_ids))
        nbytes = sum(s.nbytes for s in segs)
        if self.one_sided:
            if dst_block_ids is None or len(dst_block_ids) != len(block_ids):
                raise ValueError(f"one-sided WRITE of {rid}: {len(block_ids)} blocks but destination blocks "
                                 f"{None if dst_block_ids is None else len(dst_block_ids)}")
            x = _Xfer(rid, dst_engine, list(block_ids), segs, None, t0=time.perf_counter(),
                      meta={"dst_tp": dst_tp, "dst_blocks": list(dst_block_ids)})
            x.ids = self._ids(x.block_ids)
            x.meta["dst_ids"] = self._ids(x.meta["dst_blocks"])
        else:
            x = _Xfer(rid, dst_engine, list(block_ids), segs, self.pool.take(nbytes),
                      t0=time.perf_counter(), meta={"dst_tp": dst_tp})
            x.ids = self._ids(x.block_ids)
        self.sends[rid] = x
        self._streaming.append(x)
        self.stats["sent_bytes"] += nbytes
        self.stats["sends"] += 1
        return {"rid": rid, "nblocks": len(block_ids)}

    def _send_group(self, x: _Xfer, gi: int) -> None:
        for seg in x.segs:
            if seg.gi == gi:
                if self.one_sided:
                    self._write_seg(x, seg)
                    continue
                view = self._pack_seg(x, seg)
                x.works.append(self._track(self.links.send(x.peer, seg.piece.dst_rank, view)))
        x.packed = gi + 1

    def _write_seg(self, x: _Xfer, seg: _Seg) -> None:
        """One-sided: copy one (layer group, piece) of x's blocks into the
        decode rank's blocks on the current (copy) stream.  Every address is
        checked against the peer's layout on the host first: a bad block id
        must never become a stray write into another process's memory."""
        l0, l1 = self.groups[seg.gi]
        pc = seg.piece
        r = self.remote_kv(x.peer, pc.dst_rank)
        if r.num_layers != self.lay.num_layers:
            raise RuntimeError(f"one-sided WRITE to {x.peer}.{pc.dst_rank}: {r.num_layers} layers, "
                               f"this engine {self.lay.num_layers}")
        dst_blocks = x.meta["dst_blocks"]
        if dst_blocks and (min(dst_blocks) < 0 or max(dst_blocks) >= r.num_blocks):
            raise RuntimeError(f"one-sided WRITE of {x.rid}: destination block ids outside the peer's "
                               f"{r.num_blocks} blocks")
        if pc.dst_inner_off + pc.nbytes > r.block_bytes or pc.src_inner_off + pc.nbytes > self.lay.block_bytes:
            raise RuntimeError(f"one-sided WRITE of {x.rid}: relayout piece outside a block")
        src = self.kv[l0:l1]
        n_prefix = (l1 - l0) * 2
        dst_stride = r.num_blocks * r.block_bytes
        if r.tensor is not None:  # in-process peer (tests, CPU engines)
            ops.kv_copy_blocks(r.tensor[l0:l1], src, x.ids, x.meta["dst_ids"], n_prefix, self.lay.prefix_stride,
                               dst_stride, self.lay.block_bytes, r.block_bytes, pc.nbytes,
                               src_inner_off=pc.src_inner_off, dst_inner_off=pc.dst_inner_off)
        else:
            ops.kv_copy_blocks(src, src, x.ids, x.meta["dst_ids"], n_prefix, self.lay.prefix_stride, dst_stride,
                               self.lay.block_bytes, r.block_bytes, pc.nbytes, src_inner_off=pc.src_inner_off,
                               dst_inner_off=pc.dst_inner_off, dst_ptr=r.ptr + l0 * 2 * dst_stride)

    def on_layer(self, layer: int) -> None:
        """Model forward hook: layer `layer`'s KV is in the cache.  At the end
        of a layer group, pack + send that group of every announced request on
        the copy stream, which waits for the compute stream's progress up to
        this point only."""
        if not self._streaming:
            return
        gi = next((i for i, (l0, l1) in enumerate(self.groups) if l1 - 1 == layer), None)
        if gi is None:
            return
        ev = None
        if self.copy_stream is not None:
            ev = torch.cuda.Event()
            ev.record()
        with self._ctx():
            if ev is not None:
                self.copy_stream.wait_event(ev)
            for x in self._streaming:
                if x.packed == gi:
                    self._send_group(x, gi)

    def end_forward(self) -> None:
        """After the forward: send every group the layer hook did not reach
        (eager paths without hooks) and order the compute stream after all
        packs, so the announced requests' blocks may be reused from the next
        step on (their bytes are in staging)."""
        if not self._streaming:
            return
        if self.copy_stream is not None:
            self.copy_stream.wait_stream(torch.cuda.current_stream(self.kv.device))
        with self._ctx():
            for gi in range(len(self.groups)):  # group-major, like on_layer and the receivers
                for x in self._streaming:
                    if x.packed == gi:
                        self._send_group(x, gi)
        if self.one_sided:  # the writes of each request are complete when the copy stream passes this point
            for x in self._streaming:
                if self.copy_stream is not None:
                    x.event = torch.cuda.Event()
                    x.event.record(self.copy_stream)
                else:
                    x.event = True
        if self.copy_stream is not None:
            torch.cuda.current_stream(self.kv.device).wait_stream(self.copy_stream)
        self._streaming = []

    def poll_sends(self) -> list[str]:
        """Requests whose sends completed on this rank (staging recycled;
        one-sided: their writes landed in the peer's blocks)."""
        done = []
        for rid, x in list(self.sends.items()):
            if self.one_sided:
                if x.packed == len(self.groups) and x.event is not None and (x.event is True or x.event.query()):
                    del self.sends[rid]
                    self.stats["send_time"] += time.perf_counter() - x.t0
                    done.append(rid)
                continue
            if x.packed == len(self.groups) and all(self._done(w) for w in x.works):
                del self.sends[rid]
                self.pool.give(x.buf)
                self.stats["send_time"] += time.perf_counter() - x.t0
                done.append(rid)
        return done

    # ------------------------------------------------------------ decode side: WRITE
    def post_recv_batch(self, src_engine: str, src_tp: int, items: list[tuple]) -> None:
        """One announcement of (rid, nblocks, block_ids | None) items from one
        prefill engine, in its announcement order: post this rank's receives
        group-major, the order the prefill ranks post their sends in.
        block_ids None: the request is gone, its bytes are drained and dropped."""
        pieces = self._my(src_tp, self.tp, "dst")
        xs = []
        for rid, nblocks, block_ids in items:
            segs = self._segs(pieces, nblocks)
            nbytes = sum(s.nbytes for s in segs)
            x = _Xfer(rid, src_engine, list(block_ids) if block_ids is not None else None, segs,
                      self.pool.take(nbytes), t0=time.perf_counter())
            x.ids = self._ids(x.block_ids)
            self.recvs[rid] = x
            self.stats["recv_bytes"] += nbytes
            self.stats["recvs"] += 1
            xs.append(x)
        for gi in range(len(self.groups)):
            for x in xs:
                for seg in x.segs:
                    if seg.gi == gi:
                        view = x.buf[seg.off:seg.off + seg.nbytes]
                        x.works.append(self._track(self.links.recv(x.peer, seg.piece.src_rank, view)))

    def recvs_landed(self) -> list[str]:
        """Requests whose receives on THIS rank completed (the engine leader
        turns its own into lockstep finish events)."""
        return [rid for rid, x in self.recvs.items() if x.event is None and all(self._done(w) for w in x.works)]

    def finish_recv(self, rid: str, unpack: bool = True) -> bool:
        """Lockstep on every decode rank: unpack x into its blocks (copy
        stream after this rank's receives; compute stream after the unpack).
        unpack=False (the request was cancelled meanwhile): only drain."""
        x = self.recvs.get(rid)
        if x is None or x.event is not None:
            return False
        if not unpack:
            self.stats["dropped"] += 1
        self._unpack(x, unpack)
        self._retire(self.recvs, "recv_time")
        return True

    def poll_recvs(self) -> None:
        self._retire(self.recvs, "recv_time")

    # ------------------------------------------------------------ READ: decode side serves prefix blocks
    def serve_read(self, rid: str, block_ids: list[int], dst_engine: str, dst_tp: int = 1) -> None:
        """Lockstep on every decode rank: pack this rank's pieces of the
        cached blocks and send them to the pulling prefill engine (reverse
        links).  The decode engine is the source of the READ, so the plan is
        (decode TP -> prefill TP)."""
        segs = self._segs(self._my(self.tp, dst_tp, "src"), len(block_ids), groups=[(0, self.lay.num_layers)])
        nbytes = sum(s.nbytes for s in segs)
        x = _Xfer(rid, dst_engine, list(block_ids), segs, self.pool.take(nbytes), t0=time.perf_counter())
        x.ids = self._ids(x.block_ids)
        if self.copy_stream is not None:
            self.copy_stream.wait_stream(torch.cuda.current_stream(self.kv.device))
        with self._ctx():
            for seg in segs:
                view = x.buf[seg.off:seg.off + seg.nbytes]
                pc = seg.piece
                if self.host_staging:
                    view.copy_(pack_blocks(self.kv, x.ids, inner_off=pc.src_inner_off, inner_bytes=pc.nbytes))
                    torch.cuda.current_stream().synchronize()
                else:
                    pack_blocks(self.kv, x.ids, inner_off=pc.src_inner_off, inner_bytes=pc.nbytes, out=view)
                x.works.append(self._track(self.links.send(dst_engine, pc.dst_rank, view, rev=True)))
        self.served.append(x)
        self.stats["read_bytes"] += nbytes
        self.stats["served"] += 1

    def poll_served(self) -> int:
        while self.served and all(self._done(w) for w in self.served[0].works):
            self.pool.give(self.served.popleft().buf)
        return len(self.served)

    # ------------------------------------------------------------ READ: prefill side pulls prefix blocks
    def post_read(self, rid: str, block_ids: list[int], src_engine: str, src_tp: int = 1) -> None:
        """Lockstep on every prefill rank: post the receives of this rank's
        pieces of blocks the decode engine caches (reverse links)."""
        segs = self._segs(self._my(src_tp, self.tp, "dst"), len(block_ids), groups=[(0, self.lay.num_layers)])
        nbytes = sum(s.nbytes for s in segs)
        x = _Xfer(rid, src_engine, list(block_ids), segs, self.pool.take(nbytes),
                  t0=time.perf_counter(), meta={"read": True})
        x.ids = self._ids(x.block_ids)
        for seg in segs:
            view = x.buf[seg.off:seg.off + seg.nbytes]
            x.works.append(self._track(self.links.recv(src_engine, seg.piece.src_rank, view, rev=True)))
        self.reads_in[rid] = x
        self.stats["reads"] += 1

    def read_one_sided(self, rid: str, block_ids: list[int], src_engine: str, src_tp: int,
                       src_block_ids: list[int]) -> None:
        """One-sided READ (Patch:1296-1360's NIXL read): copy this rank's
        pieces of the decode engine's cached blocks straight from its mapped
        caches into block_ids on the copy stream.  The caller holds both
        ends' blocks until reads_landed() reports it (prefill: write_pending,
        decode: read_pinned)."""
        if len(src_block_ids) != len(block_ids):
            raise ValueError(f"one-sided READ of {rid}: {len(block_ids)} blocks, {len(src_block_ids)} sources")
        x = _Xfer(rid, src_engine, list(block_ids), [], None, t0=time.perf_counter(),
                  meta={"read": True, "one_sided": True})
        x.ids = self._ids(x.block_ids)
        src_ids = self._ids(list(src_block_ids))
        L = self.lay.num_layers
        with self._ctx():
            for pc in self._my(src_tp, self.tp, "dst"):
                r = self.remote_kv(src_engine, pc.src_rank)
                if r.num_layers != L:
                    raise RuntimeError(f"one-sided READ from {src_engine}.{pc.src_rank}: {r.num_layers} layers")
                if src_block_ids and (min(src_block_ids) < 0 or max(src_block_ids) >= r.num_blocks):
                    raise RuntimeError(f"one-sided READ of {rid}: source block ids outside the peer's "
                                       f"{r.num_blocks} blocks")
                if pc.src_inner_off + pc.nbytes > r.block_bytes or pc.dst_inner_off + pc.nbytes > self.lay.block_bytes:
                    raise RuntimeError(f"one-sided READ of {rid}: relayout piece outside a block")
                sps = r.num_blocks * r.block_bytes
                if r.tensor is not None:
                    ops.kv_copy_blocks(self.kv, r.tensor, src_ids, x.ids, L * 2, sps, self.lay.prefix_stride,
                                       r.block_bytes, self.lay.block_bytes, pc.nbytes,
                                       src_inner_off=pc.src_inner_off, dst_inner_off=pc.dst_inner_off)
                else:
                    ops.kv_copy_blocks(self.kv, self.kv, src_ids, x.ids, L * 2, sps, self.lay.prefix_stride,
                                       r.block_bytes, self.lay.block_bytes, pc.nbytes, src_inner_off=pc.src_inner_off,
                                       dst_inner_off=pc.dst_inner_off, src_ptr=r.ptr)
        if self.copy_stream is not None:
            x.meta["landed"] = torch.cuda.Event()
            x.meta["landed"].record(self.copy_stream)
        else:
            x.meta["landed"] = True
        self.reads_in[rid] = x
        self.stats["reads"] += 1
        self.stats["read_bytes"] += sum(pc.nbytes for pc in self._my(src_tp, self.tp, "dst")) * L * 2 * len(block_ids)

    def reads_landed(self) -> list[str]:
        out = []
        for rid, x in self.reads_in.items():
            if x.event is not None:
                continue
            if x.meta.get("one_sided"):
                ev = x.meta["landed"]
                if ev is True or ev.query():
                    out.append(rid)
            elif all(self._done(w) for w in x.works):
                out.append(rid)
        return out

    def finish_read(self, rid: str, unpack: bool = True) -> bool:
        """Lockstep on every prefill rank: unpack the pulled prefix (the whole
        model's layers, one segment per piece) into the request's blocks.
        unpack=False (the request was aborted meanwhile, its blocks may
        already belong to another request): only drain the receive."""
        x = self.reads_in.get(rid)
        if x is None or x.event is not None:
            return False
        if x.meta.get("one_sided"):  # the bytes are in the blocks already: order the compute stream after them
            if self.copy_stream is not None and unpack:
                torch.cuda.current_stream(self.kv.device).wait_event(x.meta["landed"])
            x.event = x.meta["landed"]
            self._retire(self.reads_in, None)
            return True
        with self._ctx():
            for w in x.works:
                self._wait(w)
            if unpack:
                for seg in x.segs:
                    src = x.buf[seg.off:seg.off + seg.nbytes]
                    FAULTS.corrupt_received(src)
                    if self.host_staging:
                        src = src.to(self.kv.device, non_blocking=True)
                    unpack_blocks(self.kv, src, x.ids, inner_off=seg.piece.dst_inner_off,
                                  inner_bytes=seg.piece.nbytes)
        if self.copy_stream is not None:
            x.event = torch.cuda.Event()
            x.event.record(self.copy_stream)
            if unpack:
                torch.cuda.current_stream(self.kv.device).wait_event(x.event)
        else:
            x.event = True
        if not unpack:
            self.stats["dropped"] += 1
        self._retire(self.reads_in, None)
        return True

    def poll_reads(self) -> None:
        self._retire(self.reads_in, None)

    def pending(self) -> int:
        return len(self.sends) + len(self.recvs) + len(self.reads_in) + len(self.served)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
