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


@dataclass
class _Send:
    rid: str
    work: object
    buf: torch.Tensor
    t0: float


@dataclass
class _Recv:
    rid: str
    work: object
    buf: torch.Tensor
    block_ids: list[int]
    meta: dict
    t0: float


class RcclKVTransfer:
    """Owns outstanding RCCL sends/recvs of KV payloads for one rank."""

    def __init__(self, kv_cache: torch.Tensor, group=None, host_staging: bool = False):
        self.kv = kv_cache
        self.group = group
        # host_staging: move payloads through host memory over a gloo group
        # (single-GPU functional testing of the disagg path; not the fast path)
        self.host_staging = host_staging
        self.sends: collections.deque[_Send] = collections.deque()
        self.recvs: collections.deque[_Recv] = collections.deque()
        self.stats = dict(sent_bytes=0, recv_bytes=0, sends=0, recvs=0, send_time=0.0, recv_time=0.0)
        # gloo (CPU CI path) p2p work never reports completion by polling; its
        # wait() is short once the peer has posted (notify precedes the send)
        self.blocking = (not kv_cache.is_cuda) or host_staging

    def _done(self, work) -> bool:
        if self.blocking:
            work.wait()
            return True
        return work.is_completed()

    # ------------------------------------------------------------ prefill side
    def send(self, rid: str, block_ids: list[int], dst: int) -> int:
        import torch.distributed as dist

        buf = pack_blocks(self.kv, block_ids)
        if self.host_staging:
            buf = buf.cpu()
        work = dist.isend(buf, dst, group=self.group)
        self.sends.append(_Send(rid, work, buf, time.perf_counter()))
        self.stats["sent_bytes"] += buf.numel()
        self.stats["sends"] += 1
        return buf.numel()

    def poll_sends(self) -> list[str]:
        done = []
        while self.sends and self._done(self.sends[0].work):
            s = self.sends.popleft()
            self.stats["send_time"] += time.perf_counter() - s.t0
            done.append(s.rid)
        return done

    # ------------------------------------------------------------ decode side
    def post_recv(self, rid: str, src: int, nbytes: int, block_ids: list[int], meta: dict) -> None:
        import torch.distributed as dist

        buf = torch.empty(nbytes, dtype=torch.uint8, device="cpu" if self.host_staging else self.kv.device)
        work = dist.irecv(buf, src, group=self.group)
        self.recvs.append(_Recv(rid, work, buf, block_ids, meta, time.perf_counter()))
        self.stats["recv_bytes"] += nbytes
        self.stats["recvs"] += 1

    def poll_recvs(self) -> list[tuple[str, dict]]:
        """Unpack every completed receive (in order); returns [(rid, meta)]."""
        done = []
        while self.recvs and self._done(self.recvs[0].work):
            r = self.recvs.popleft()
            if not self.blocking:
                r.work.wait()  # orders the compute stream after the RCCL stream
            unpack_blocks(self.kv, r.buf.to(self.kv.device) if self.host_staging else r.buf, r.block_ids)
            self.stats["recv_time"] += time.perf_counter() - r.t0
            done.append((r.rid, r.meta))
        return done

    def pending(self) -> int:
        return len(self.sends) + len(self.recvs)


def init_pair_comms(rank: int, prefill_ranks: list[int], decode_ranks: list[int], device, group=None) -> None:
    """Create every prefill->decode RCCL p2p communicator up front (lazy creation
    inside the serving loop would block a rank until its peer also sends)."""
    import torch.distributed as dist

    t = torch.zeros(1, device=device)
    for p in prefill_ranks:
        for d in decode_ranks:
            if rank == p:
                dist.send(t, d, group=group)
            elif rank == d:
                dist.recv(t, p, group=group)
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
