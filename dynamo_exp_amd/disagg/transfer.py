"""Prefill -> decode KV block transfer over RCCL (xGMI), the NIXL role.

Reference behaviour: the prefill worker writes the
computed KV blocks into the decode worker's pre-allocated blocks and notifies
completion; an alternative pipe uses NCCL send/recv.  MI355X design:

  prefill rank                                   decode rank
  ------------                                   -----------
  pack blocks[skip:] of all layers (K and V)     (blocks allocated at admission)
    into one contiguous staging buffer with
    the kv_copy HIP kernel (one launch)
  notify {rid, src, nbytes, first_token}  --->   on notify: irecv(staging, src)
  isend(staging, dst) on the RCCL stream  ===>   (RCCL stream, overlaps compute)
                                                 on completion: unpack into its
                                                 blocks[skip:] (one kernel),
                                                 request joins the decode batch

Control messages go over the control plane; only bulk bytes use RCCL, in one
direction per pair, so the per-pair RCCL stream never interleaves opposing
sends and recvs (which would deadlock its in-order execution).  Messages are
posted in notification order on both sides, matching NCCL's per-peer
ordering.  One transfer per request moves all layers (~375 MiB for an 8B
3000-token prompt) as a single RCCL message (per-link bound ~ one xGMI link).

TP mismatch (decode TP = d x prefill TP): the cache layout [NB][Hkv][BS][D]
makes each decode rank's KV-head slice a contiguous sub-range of every block,
so the pack kernel's inner offset does the relayout (kv_rearrange.py analog).
"""
from __future__ import annotations

import collections
import logging
import time
from dataclasses import dataclass, field

import torch

from .. import ops

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
    decode rank (reference block_copy.cu:558-758 permute_scatter and the
    Triton kv_rearrange kernels).  With the [NB][Hkv][BS][D] block layout a
    rank's heads are one contiguous range of every block, so every piece is a
    (src offset, dst offset, length) triple the pack/unpack kernel applies to
    all blocks and layers in one launch.  Each decode rank takes every head it
    holds from the first prefill rank holding it (replicated heads when a TP
    size exceeds the KV head count); pieces are in ascending head order, the
    order both sides post their sends / receives in."""
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


def pack_blocks(kv_cache: torch.Tensor, block_ids: list[int], inner_off: int = 0, inner_bytes: int | None = None,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """Gather blocks (all layers, K and V) into [L*2, n, inner] bytes."""
    lay = KVLayout.of(kv_cache)
    n = len(block_ids)
    inner = inner_bytes or lay.block_bytes
    if out is None:
        out = torch.empty(lay.prefix * n * inner, dtype=torch.uint8, device=kv_cache.device)
    dev = kv_cache.device
    src_ids = torch.tensor(block_ids, dtype=torch.int32, device=dev)
    dst_ids = torch.arange(n, dtype=torch.int32, device=dev)
    ops.kv_copy_blocks(out, kv_cache, src_ids, dst_ids, lay.prefix, lay.prefix_stride, n * inner, lay.block_bytes,
                       inner, inner, src_inner_off=inner_off)
    return out


def unpack_blocks(kv_cache: torch.Tensor, staging: torch.Tensor, block_ids: list[int], inner_off: int = 0,
                  inner_bytes: int | None = None) -> None:
    lay = KVLayout.of(kv_cache)
    n = len(block_ids)
    inner = inner_bytes or lay.block_bytes
    dev = kv_cache.device
    src_ids = torch.arange(n, dtype=torch.int32, device=dev)
    dst_ids = torch.tensor(block_ids, dtype=torch.int32, device=dev)
    ops.kv_copy_blocks(kv_cache, staging, src_ids, dst_ids, lay.prefix, n * inner, lay.prefix_stride, inner,
                       lay.block_bytes, inner, dst_inner_off=inner_off)


def transfer_bytes(kv_cache: torch.Tensor, n_blocks: int) -> int:
    lay = KVLayout.of(kv_cache)
    return lay.prefix * n_blocks * lay.block_bytes


class StagingPool:
    """Reusable staging buffers for KV transfers (device memory, or pinned host
    memory for host-staged transport), in size classes of `granule` bytes, so
    a 3000-token Llama-3-8B request does not allocate ~375 MiB per transfer on
    each side.  A buffer goes back to the pool only after every stream that
    used it is done with it (the caller's completion event / work).  `cap`
    bounds what the pool keeps; `can_take` is the sender's backpressure test."""

    def __init__(self, device, cap_bytes: int = 4 << 30, granule: int = 8 << 20, pinned: bool = False):
        self.device = torch.device(device)
        self.cap = cap_bytes
        self.granule = granule
        self.pinned = pinned
        self.free: dict[int, list[torch.Tensor]] = collections.defaultdict(list)
        self.in_use = 0
        self.held = 0  # bytes owned by the pool (free + in use)
        self.stats = dict(allocs=0, reuses=0)

    def _cls(self, nbytes: int) -> int:
        return max(self.granule, -(-nbytes // self.granule) * self.granule)

    def can_take(self, nbytes: int) -> bool:
        c = self._cls(nbytes)
        return bool(self.free.get(c)) or self.in_use + c <= self.cap

    def take(self, nbytes: int) -> torch.Tensor:
        c = self._cls(nbytes)
        lst = self.free.get(c)
        if lst:
            buf = lst.pop()
            self.stats["reuses"] += 1
        else:
            if self.pinned:
                buf = torch.empty(c, dtype=torch.uint8).pin_memory()
            else:
                buf = torch.empty(c, dtype=torch.uint8, device=self.device)
            self.held += c
            self.stats["allocs"] += 1
        self.in_use += c
        return buf

    def give(self, buf: torch.Tensor) -> None:
        c = buf.numel()
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


@dataclass
class _Stream:
    """One request's KV moving in layer groups (either direction)."""

    rid: str
    peer: int
    block_ids: list[int]
    buf: torch.Tensor | None  # pooled staging (base tensor)
    works: list = field(default_factory=list)  # per group: [work, done]
    packed: int = 0  # groups packed + posted (sender)
    meta: dict = field(default_factory=dict)
    t0: float = 0.0
    event: object = None  # unpack completion (receiver)
    done_msg: dict | None = None  # receiver: the sender's "done" (first token)


class RcclKVTransfer:
    """KV block movement between a prefill and a decode rank over RCCL (xGMI):
    the NIXL data plane of the reference.

    * WRITE (prefill -> decode), layer-streamed: the prefill rank announces a
      request before the forward pass that completes its prompt
      (`begin_send`); after the KV of each layer group is written
      (`on_layer`, called from the model's forward) the group is packed on a
      dedicated copy stream -- which waits only for that layer's event, so the
      remaining layers keep computing -- and sent; the decode rank posts the
      group receives when the announcement arrives, so the transfer overlaps
      the rest of the prefill (reference CopyStream/trigger_layer,
      lib/llm/src/kv/layer.rs:785-1130).
    * READ (decode -> prefill): a prefill rank that lacks a prompt prefix the
      decode rank already holds pulls those blocks before computing the rest
      (reference Patch:1296-1360 read_blocks): `serve_read` on the decode side,
      `post_read` / `poll_reads` on the prefill side, on a separate process
      group so opposite directions never share an in-order RCCL stream.
    * Staging is pooled (StagingPool) and packing/unpacking run on the copy
      stream; the compute stream waits on an event only where it reads
      unpacked blocks.
    """

    def __init__(self, kv_cache: torch.Tensor, group=None, host_staging: bool = False, rev_group=None,
                 layer_group_count: int = 4, pool_cap_bytes: int = 4 << 30):
        self.kv = kv_cache
        self.group = group
        self.rev_group = rev_group if rev_group is not None else group
        # host_staging: move payloads through host memory over a gloo group
        # (single-GPU functional testing of the disagg path; not the fast path)
        self.host_staging = host_staging
        self.gpu = kv_cache.is_cuda
        self.lay = KVLayout.of(kv_cache)
        self.groups = layer_groups(self.lay.num_layers, layer_group_count)
        self.copy_stream = torch.cuda.Stream(kv_cache.device) if self.gpu else None
        self.pool = StagingPool("cpu" if (host_staging or not self.gpu) else kv_cache.device, pool_cap_bytes,
                                pinned=host_staging and self.gpu)
        self.sends: dict[str, _Stream] = {}
        self.recvs: dict[str, _Stream] = {}
        self.reads_out: dict[str, _Stream] = {}  # decode side: prefix blocks being served
        self.reads_in: dict[str, _Stream] = {}  # prefill side: prefix blocks being pulled
        self._streaming: list[_Stream] = []  # sends announced for the current forward
        self.stats = dict(sent_bytes=0, recv_bytes=0, sends=0, recvs=0, send_time=0.0, recv_time=0.0,
                          read_bytes=0, reads=0)
        # gloo (CPU CI path) p2p work never reports completion by polling; its
        # wait() is short once the peer has posted (announcements precede sends)
        self.blocking = (not self.gpu) or host_staging

    # ------------------------------------------------------------ helpers
    def group_bytes(self, nblocks: int) -> list[int]:
        return [(l1 - l0) * 2 * nblocks * self.lay.block_bytes for l0, l1 in self.groups]

    def _done(self, w: list) -> bool:
        # gloo's wait() on a receive waits for the NEXT message each call, so a
        # completed work is never waited on again
        if not w[1]:
            if self.blocking:
                w[0].wait()
                w[1] = True
            else:
                w[1] = w[0].is_completed()
        return w[1]

    def _ctx(self):
        return torch.cuda.stream(self.copy_stream) if self.copy_stream is not None else _nullctx()

    def _pack_into(self, dst: torch.Tensor, block_ids: list[int], l0: int, l1: int) -> torch.Tensor:
        """Pack layers [l0, l1) of block_ids into dst (device) on the current stream."""
        return pack_blocks(self.kv[l0:l1], block_ids, out=dst)

    def _wire(self, buf: torch.Tensor, nbytes: int, off: int = 0) -> torch.Tensor:
        return buf[off:off + nbytes]

    def _send_group(self, st: _Stream, gi: int, group) -> None:
        import torch.distributed as dist

        l0, l1 = self.groups[gi]
        nb = self.group_bytes(len(st.block_ids))
        off = sum(nb[:gi])
        view = self._wire(st.buf, nb[gi], off)
        if self.host_staging:  # pack on the device, then through pinned host memory
            tmp = self._pack_into(torch.empty(nb[gi], dtype=torch.uint8, device=self.kv.device), st.block_ids, l0, l1)
            view.copy_(tmp)
            if self.copy_stream is not None:
                torch.cuda.current_stream().synchronize()
        else:
            self._pack_into(view, st.block_ids, l0, l1)
        st.works.append([dist.isend(view, st.peer, group=group), False])

    # ------------------------------------------------------------ prefill side: WRITE
    def begin_send(self, rid: str, block_ids: list[int], dst: int) -> dict:
        """Announce a request whose prompt completes in the coming forward;
        returns the announcement the decode rank needs to post its receives."""
        nb = self.group_bytes(len(block_ids))
        st = _Stream(rid, dst, list(block_ids), self.pool.take(sum(nb)), t0=time.perf_counter())
        self.sends[rid] = st
        self._streaming.append(st)
        self.stats["sent_bytes"] += sum(nb)
        self.stats["sends"] += 1
        return {"rid": rid, "nblocks": len(block_ids), "groups": len(self.groups), "nbytes": sum(nb)}

    def on_layer(self, layer: int) -> None:
        """Model forward hook: layer `layer`'s KV is in the cache.  At the end
        of a layer group, pack + send that group of every announced request
        on the copy stream (which waits for the compute stream's progress up
        to this point only)."""
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
            for st in self._streaming:
                if st.packed == gi:
                    self._send_group(st, gi, self.group)
                    st.packed += 1

    def end_forward(self) -> None:
        """After the forward: send any group the hook did not reach (eager
        paths without layer hooks) and close the announcement list."""
        if self._streaming and self.copy_stream is not None:
            self.copy_stream.wait_stream(torch.cuda.current_stream())
        with self._ctx():
            for gi in range(len(self.groups)):  # group-major, like on_layer and the receivers
                for st in self._streaming:
                    if st.packed == gi:
                        self._send_group(st, gi, self.group)
                        st.packed += 1
        self._streaming = []

    def send(self, rid: str, block_ids: list[int], dst: int) -> int:
        """Whole-request send after the fact (no layer hook): announce + send."""
        m = self.begin_send(rid, block_ids, dst)
        self.end_forward()
        return m["nbytes"]

    def poll_sends(self) -> list[str]:
        done = []
        for rid, st in list(self.sends.items()):
            if st.packed == len(self.groups) and all(self._done(w) for w in st.works):
                del self.sends[rid]
                self.pool.give(st.buf)
                self.stats["send_time"] += time.perf_counter() - st.t0
                done.append(rid)
        return done

    # ------------------------------------------------------------ decode side: WRITE
    def post_recv(self, rid: str, src: int, nblocks: int, block_ids: list[int] | None, meta: dict) -> None:
        self.post_recv_batch(src, [(rid, nblocks, block_ids, meta)])

    def post_recv_batch(self, src: int, items: list[tuple]) -> None:
        """On an announcement of (rid, nblocks, block_ids | None, meta) items
        from one prefill rank, in its announcement order: post the receives
        group-major -- group 0 of every item, then group 1, ... -- the order
        that rank posts its sends in (on_layer / end_forward), since RCCL
        matches point-to-point messages of a pair strictly in order.
        block_ids None: the request is gone, its bytes are drained and dropped."""
        import torch.distributed as dist

        sts = []
        for rid, nblocks, block_ids, meta in items:
            nb = self.group_bytes(nblocks)
            st = _Stream(rid, src, list(block_ids) if block_ids is not None else None, self.pool.take(sum(nb)),
                         meta=dict(meta, nblocks=nblocks), t0=time.perf_counter())
            self.recvs[rid] = st
            self.stats["recv_bytes"] += sum(nb)
            self.stats["recvs"] += 1
            sts.append((st, nb))
        for gi in range(len(self.groups)):
            for st, nb in sts:
                off = sum(nb[:gi])
                st.works.append([dist.irecv(self._wire(st.buf, nb[gi], off), src, group=self.group), False])

    def sender_done(self, rid: str, msg: dict) -> None:
        """The sender's completion message (first token / logprob)."""
        st = self.recvs.get(rid)
        if st is not None:
            st.done_msg = msg

    def poll_recvs(self) -> list[tuple[str, dict]]:
        """Requests whose every group landed and whose first token arrived:
        unpack (copy stream), order the compute stream after the unpack, and
        return [(rid, meta + done message)]."""
        out = []
        for rid, st in list(self.recvs.items()):
            if st.done_msg is None or st.event is not None:
                continue
            if not all(self._done(w) for w in st.works):
                continue
            self._unpack(st)
            out.append((rid, {**st.meta, **st.done_msg}))
        self._retire(self.recvs, "recv_time")
        return out

    def _unpack(self, st: _Stream) -> None:
        if st.block_ids is not None:
            nb = self.group_bytes(len(st.block_ids))
            with self._ctx():
                for w in st.works:
                    if self.gpu and not self.blocking:
                        w[0].wait()  # the copy stream waits for the RCCL stream (no host block)
                off = 0
                for (l0, l1), n in zip(self.groups, nb):
                    src = self._wire(st.buf, n, off)
                    if self.host_staging:
                        src = src.to(self.kv.device, non_blocking=True)
                    unpack_blocks(self.kv[l0:l1], src, st.block_ids)
                    off += n
        if self.copy_stream is not None:
            st.event = torch.cuda.Event()
            st.event.record(self.copy_stream)
            torch.cuda.current_stream(self.kv.device).wait_event(st.event)  # readers of the blocks wait
        else:
            st.event = True

    def _retire(self, table: dict, timer: str | None) -> None:
        """Give staging back once its unpack finished."""
        for rid, st in list(table.items()):
            if st.event is None:
                continue
            if st.event is True or st.event.query():
                del table[rid]
                self.pool.give(st.buf)
                if timer:
                    self.stats[timer] += time.perf_counter() - st.t0

    # ------------------------------------------------------------ READ: decode side serves prefix blocks
    def serve_read(self, rid: str, block_ids: list[int], dst: int) -> None:
        import torch.distributed as dist

        nbytes = self.lay.prefix * len(block_ids) * self.lay.block_bytes
        st = _Stream(rid, dst, list(block_ids), self.pool.take(nbytes), t0=time.perf_counter())
        if self.copy_stream is not None:
            self.copy_stream.wait_stream(torch.cuda.current_stream())
        with self._ctx():
            view = self._wire(st.buf, nbytes)
            if self.host_staging:
                view.copy_(pack_blocks(self.kv, block_ids))
                torch.cuda.current_stream().synchronize()
            else:
                pack_blocks(self.kv, block_ids, out=view)
            st.works.append([dist.isend(view, dst, group=self.rev_group), False])
        self.reads_out[rid] = st
        self.stats["read_bytes"] += nbytes

    def poll_served_reads(self) -> int:
        for rid, st in list(self.reads_out.items()):
            if all(self._done(w) for w in st.works):
                del self.reads_out[rid]
                self.pool.give(st.buf)
        return len(self.reads_out)

    # ------------------------------------------------------------ READ: prefill side pulls prefix blocks
    def post_read(self, rid: str, src: int, block_ids: list[int]) -> None:
        import torch.distributed as dist

        nbytes = self.lay.prefix * len(block_ids) * self.lay.block_bytes
        st = _Stream(rid, src, list(block_ids), self.pool.take(nbytes), t0=time.perf_counter())
        st.works.append([dist.irecv(self._wire(st.buf, nbytes), src, group=self.rev_group), False])
        self.reads_in[rid] = st
        self.stats["reads"] += 1

    def poll_reads(self) -> list[str]:
        """Pulled prefixes that landed: unpack into the request's blocks and
        return their request ids (the scheduler resumes them)."""
        out = []
        for rid, st in list(self.reads_in.items()):
            if st.event is not None or not all(self._done(w) for w in st.works):
                continue
            nbytes = self.lay.prefix * len(st.block_ids) * self.lay.block_bytes
            with self._ctx():
                if self.gpu and not self.blocking:
                    st.works[0][0].wait()
                src = self._wire(st.buf, nbytes)
                if self.host_staging:
                    src = src.to(self.kv.device, non_blocking=True)
                unpack_blocks(self.kv, src, st.block_ids)
            if self.copy_stream is not None:
                st.event = torch.cuda.Event()
                st.event.record(self.copy_stream)
                torch.cuda.current_stream(self.kv.device).wait_event(st.event)
            else:
                st.event = True
            out.append(rid)
        self._retire(self.reads_in, None)
        return out

    def pending(self) -> int:
        return len(self.sends) + len(self.recvs) + len(self.reads_out) + len(self.reads_in)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def init_pair_comms(rank: int, prefill_ranks: list[int], decode_ranks: list[int], device, group=None,
                    rev_group=None) -> None:
    """Create every prefill->decode RCCL p2p communicator (and the decode->
    prefill ones of `rev_group`) up front: lazy creation inside the serving
    loop would block a rank until its peer also sends."""
    import torch.distributed as dist

    t = torch.zeros(1, device=device)
    for p in prefill_ranks:
        for d in decode_ranks:
            if rank == p:
                dist.send(t, d, group=group)
                if rev_group is not None:
                    dist.recv(t, d, group=rev_group)
            elif rank == d:
                dist.recv(t, p, group=group)
                if rev_group is not None:
                    dist.send(t, p, group=rev_group)
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
