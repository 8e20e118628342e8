"""Custom all-reduce over xGMI peer memory for TP messages (SURVEY §2.14:
"custom one-shot/two-shot all-reduce writing to peers' buffers over all 7
xGMI links"; the reference delegates this to vLLM's custom all-reduce inside
its engines).

Every rank registers one input buffer (torch CUDA storage shared through its
IPC handle) and one signal array (uncached device memory, raw IPC handle).
`all_reduce(x)` launches `csrc/kernels/custom_ar.hip`:

* one-shot (messages <= `one_shot_max`, decode sizes): every rank reads the
  whole message from every peer over its direct link and sums in fp32;
* two-shot (larger, up to the buffer size, prefill sizes): reduce-scatter in
  place in the registered buffers, then all-gather -- each rank moves
  2(N-1)/N of the message, spread over its N-1 links.

The input normally lands in the registered buffer straight from the
producing GEMM (`buffer()` hands out a view of it; `TPGroup.rowparallel_mm`
writes the O / down projection there), so no copy precedes the kernel; other
inputs are copied in first.  The kernel counts its call index on the device
(graph-capturable: every replay gets a fresh barrier epoch).  A peer that
does not arrive within the spin limit makes the kernel set an error flag and
return without touching data; `check()` (called after every engine step by
the TP driver) turns that into a worker failure instead of wrong tokens.

Used by `TPGroup` by default for bf16 messages up to the buffer size
(DX_CUSTOM_AR=0 disables it: RCCL all-reduce for everything).

Failure model.  The error flag is sticky on the device: once a barrier of
this rank timed out (DX_CUSTOM_AR_TIMEOUT_MS, default 20 s), every later
launch returns at entry without touching data, so a captured decode graph
with dozens of collectives fails in one timeout instead of one per launch.

Ranks that share ONE device (functional rehearsals with several TP ranks on
a one-GPU box) do not get the custom all-reduce unless DX_CUSTOM_AR_SHARED=1:
its spin barrier needs the peer's kernel to be resident at the same time,
and kernels of different processes on one GPU are time-sliced by the
hardware scheduler, not co-scheduled -- with four processes on one GPU a
barrier was starved past its timeout (round 4,
profiles/r4_tp2_rehearsal_test_hang.log: the prefill follower blocked in a
host sync behind its own compute stream while the leader waited for it in
the next collective).  `create()` returns None for such a group, and the TP
group falls back to torch.distributed.
"""
from __future__ import annotations

import os

import torch

from .. import _native


def timeout_ms() -> int:
    return int(os.environ.get("DX_CUSTOM_AR_TIMEOUT_MS", "0") or 0)


class _Endpoint:
    """One rank's view: own buffer/signals + peer pointers."""

    def __init__(self, rank: int, world: int, buf: torch.Tensor, buf_ptrs: list[int], sig_ptrs: list[int]):
        self.rank, self.world = rank, world
        self.buf = buf
        self.buf_ptrs, self.sig_ptrs = buf_ptrs, sig_ptrs
        self.err = torch.zeros(1, dtype=torch.int32, device=buf.device)


class CustomAllReduce:
    ONE_SHOT_MAX = 1 << 20  # bytes; above: two-shot

    def __init__(self, endpoint: _Endpoint, max_bytes: int, one_shot_blocks: int = 32, two_shot_blocks: int = 64,
                 owned: list | None = None):
        self.ep = endpoint
        self.max_bytes = max_bytes
        self.one_shot_max = min(self.ONE_SHOT_MAX, max_bytes)
        self.one_shot_blocks, self.two_shot_blocks = one_shot_blocks, two_shot_blocks
        self._owned = owned or []  # (kind, ptr) to release
        self.timeout_ms = timeout_ms()

    # ---------------------------------------------------------------- setup
    @classmethod
    def create(cls, group, rank: int, world: int, device: torch.device, max_bytes: int = 64 << 20):
        """Collective over `group` (torch.distributed): allocate, exchange
        IPC handles, open peers.  Returns None (on every rank alike) when two
        ranks share one device, unless DX_CUSTOM_AR_SHARED=1."""
        import torch.distributed as dist

        ids: list = [None] * world
        dist.all_gather_object(ids, device_identity(device), group=group)
        if len(set(ids)) < world and os.environ.get("DX_CUSTOM_AR_SHARED", "0") in ("", "0"):
            return None
        k = _native.kernels()
        buf = torch.empty(max_bytes, dtype=torch.uint8, device=device)
        sig = k.custom_ar_alloc_signals()
        # shared by our own IPC handle of the buffer's allocation (+ offset),
        # not torch's CUDA-tensor sharing: no producer/consumer reference
        # counting to outlive, and every mapping is closed by close()
        base, off = k.alloc_base_offset(buf.data_ptr())
        mine = {"rank": rank, "buf": k.ipc_get_handle(base), "off": off, "sig": k.ipc_get_handle(sig)}
        allv: list = [None] * world
        dist.all_gather_object(allv, mine, group=group)
        buf_ptrs, sig_ptrs, owned = [], [], [("dev", sig)]
        for r, m in enumerate(allv):
            if r == rank:
                buf_ptrs.append(buf.data_ptr())
                sig_ptrs.append(sig)
                continue
            pb = k.ipc_open_handle(m["buf"])
            owned.append(("ipc", pb))
            buf_ptrs.append(pb + m["off"])
            p = k.ipc_open_handle(m["sig"])
            owned.append(("ipc", p))
            sig_ptrs.append(p)
        return cls(_Endpoint(rank, world, buf, buf_ptrs, sig_ptrs), max_bytes, owned=owned)

    @classmethod
    def local_ranks(cls, world: int, device: torch.device, max_bytes: int = 1 << 20) -> list["CustomAllReduce"]:
        """`world` virtual ranks on ONE device (tests the protocol and the
        kernel without a multi-GPU node)."""
        k = _native.kernels()
        bufs = [torch.empty(max_bytes, dtype=torch.uint8, device=device) for _ in range(world)]
        sigs = [k.custom_ar_alloc_signals() for _ in range(world)]
        ptrs = [b.data_ptr() for b in bufs]
        return [cls(_Endpoint(r, world, bufs[r], ptrs, sigs), max_bytes, owned=[("dev", sigs[r])])
                for r in range(world)]

    def close(self) -> None:
        k = _native.kernels()
        torch.cuda.synchronize(self.ep.buf.device)  # no kernel of ours still reads a peer buffer
        for kind, p in self._owned:
            (k.ipc_close_handle if kind == "ipc" else k.device_free)(p)
        self._owned = []
        self.ep.buf_ptrs = [self.ep.buf.data_ptr()]

    # ---------------------------------------------------------------- use
    def should_use(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return x.dtype == torch.bfloat16 and x.is_contiguous() and n <= self.max_bytes and x.numel() % 8 == 0

    def fits(self, shape, dtype=torch.bfloat16) -> bool:
        n = 1
        for d in shape:
            n *= d
        return dtype == torch.bfloat16 and n % 8 == 0 and n * 2 <= self.max_bytes

    def buffer(self, shape, dtype=torch.bfloat16) -> torch.Tensor:
        """A [shape] view at the start of this rank's registered buffer: a
        producer that writes its output here saves the input copy."""
        n = 1
        for d in shape:
            n *= d
        return self.ep.buf[: n * torch.tensor([], dtype=dtype).element_size()].view(dtype).view(*shape)

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        ep = self.ep
        n = x.numel()
        nbytes = n * x.element_size()
        if x.data_ptr() != ep.buf.data_ptr():
            ep.buf[:nbytes].copy_(x.view(-1).view(torch.uint8))
            out = x if out is None else out
        elif out is None:
            out = torch.empty_like(x)  # the buffer itself is scratch for the next call
        two = nbytes > self.one_shot_max
        st = stream if stream is not None else torch.cuda.current_stream(x.device)
        _native.kernels().custom_ar(out.data_ptr(), ep.buf_ptrs, ep.sig_ptrs, ep.rank, ep.world, n, self.timeout_ms,
                                    self.two_shot_blocks if two else self.one_shot_blocks, ep.err.data_ptr(),
                                    int(two), st.cuda_stream)
        return out

    def fits_gather(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return x.is_contiguous() and -(-n // 16) * 16 <= self.max_bytes

    def all_gather(self, x: torch.Tensor, stream=None) -> torch.Tensor:
        """[*s] on every rank -> [world, *s] (rank order), every peer's share
        read over its own link (csrc/kernels/custom_ar.hip custom_ag).
        Messages are moved in 16-B vectors, padded (e.g. the sampler's
        [B, 5] fp32 partials at odd B).  Graph-capturable; same barrier
        sequence as the all-reduces."""
        ep = self.ep
        nbytes = x.numel() * x.element_size()
        pb = -(-nbytes // 16) * 16
        if x.data_ptr() != ep.buf.data_ptr():
            ep.buf[:nbytes].copy_(x.reshape(-1).view(torch.uint8))
        raw = torch.empty(ep.world * pb, dtype=torch.uint8, device=x.device)
        st = stream if stream is not None else torch.cuda.current_stream(x.device)
        _native.kernels().custom_ag(raw.data_ptr(), ep.buf_ptrs, ep.sig_ptrs, ep.rank, ep.world, pb,
                                    self.one_shot_blocks, ep.err.data_ptr(), self.timeout_ms, st.cuda_stream)
        rows = raw.view(ep.world, pb)
        if pb != nbytes:
            rows = rows[:, :nbytes].contiguous()
        return rows.view(x.dtype).view((ep.world,) + tuple(x.shape))

    def check(self, blocking: bool = False) -> None:
        """Raise if any launch so far saw a peer miss its barrier.  Non-blocking
        by default (called after every engine step with the next batch already
        in flight under asynchronous scheduling): the flag is copied to pinned
        host memory on the stream and inspected once that copy has completed,
        i.e. a failure surfaces one or two steps later instead of stalling the
        host on the GPU every step."""
        ep = self.ep
        if blocking:
            if int(ep.err.item()):
                raise RuntimeError("custom all-reduce: a peer did not arrive (barrier timeout); results are invalid")
            return
        if getattr(self, "_err_host", None) is None:
            self._err_host = torch.zeros(1, dtype=torch.int32).pin_memory()
            self._err_ev = None
        ev = self._err_ev
        if ev is not None:
            if not ev.query():
                return  # the previous copy is still queued behind the step
            if int(self._err_host[0]):
                raise RuntimeError("custom all-reduce: a peer did not arrive (barrier timeout); results are invalid")
        self._err_host.copy_(ep.err, non_blocking=True)
        self._err_ev = torch.cuda.Event()
        self._err_ev.record()


def device_identity(device: torch.device) -> str:
    """Physical identity of a device (PCI location, else UUID): equal for
    two processes that see the same GPU under different indices."""
    p = torch.cuda.get_device_properties(device)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}/{p.uuid}"


def enabled() -> bool:
    return os.environ.get("DX_CUSTOM_AR", "1") not in ("", "0")
