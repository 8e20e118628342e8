"""One-shot custom all-reduce over xGMI for small TP messages (SURVEY §2.14:
"custom one-shot/two-shot all-reduce writing to peers' buffers over all 7
xGMI links for decode-size messages"; the reference delegates this to vLLM's
custom all-reduce inside its engines).

Every rank registers one input buffer (torch CUDA storage shared through its
IPC handle) and one signal array (uncached device memory, raw IPC handle);
`all_reduce(x)` copies x into the own buffer and launches the one-shot kernel
(`csrc/kernels/custom_ar.hip`), which reads all peers' buffers over their
direct links and writes the fp32-accumulated sum.  Used by `TPGroup` for
messages up to `max_bytes` when enabled (DX_CUSTOM_AR=1); larger messages and
the default path use RCCL all-reduce.  The kernel is graph-capturable (the
per-call epoch lives in a device counter bumped by the kernel launch wrapper
on the host, so capture is only used with a fixed replay order).
"""
from __future__ import annotations

import os

import torch

from .. import _native


class _Endpoint:
    """One rank's view: own buffer/signals + peer pointers."""

    def __init__(self, rank: int, world: int, buf: torch.Tensor, buf_ptrs: list[int], sig_ptrs: list[int]):
        self.rank, self.world = rank, world
        self.buf = buf
        self.buf_ptrs, self.sig_ptrs = buf_ptrs, sig_ptrs
        self.err = torch.zeros(1, dtype=torch.int32, device=buf.device)
        self.epoch = 0


class CustomAllReduce:
    def __init__(self, endpoint: _Endpoint, max_bytes: int, blocks: int = 32, owned: list | None = None):
        self.ep = endpoint
        self.max_bytes = max_bytes
        self.blocks = blocks
        self._owned = owned or []  # (kind, ptr) to release

    # ---------------------------------------------------------------- setup
    @classmethod
    def create(cls, group, rank: int, world: int, device: torch.device, max_bytes: int = 4 << 20):
        """Collective over `group` (torch.distributed): allocate, exchange
        IPC handles, open peers."""
        import torch.distributed as dist

        k = _native.kernels()
        buf = torch.empty(max_bytes, dtype=torch.uint8, device=device)
        sig = k.custom_ar_alloc_signals()
        st = buf.untyped_storage()
        handle = st._share_cuda_()
        offset = buf.storage_offset()
        mine = {"rank": rank, "buf": handle, "off": offset, "sig": k.ipc_get_handle(sig)}
        allv: list = [None] * world
        dist.all_gather_object(allv, mine, group=group)
        buf_ptrs, sig_ptrs, owned, keep = [], [], [("dev", sig)], []
        for r, m in enumerate(allv):
            if r == rank:
                buf_ptrs.append(buf.data_ptr())
                sig_ptrs.append(sig)
                continue
            peer_storage = torch.UntypedStorage._new_shared_cuda(*m["buf"])
            keep.append(peer_storage)
            buf_ptrs.append(peer_storage.data_ptr() + m["off"])
            p = k.ipc_open_handle(m["sig"])
            owned.append(("ipc", p))
            sig_ptrs.append(p)
        ar = cls(_Endpoint(rank, world, buf, buf_ptrs, sig_ptrs), max_bytes, owned=owned)
        ar._keep = keep
        return ar

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
        for kind, p in self._owned:
            (k.ipc_close_handle if kind == "ipc" else k.device_free)(p)
        self._owned = []

    # ---------------------------------------------------------------- use
    def should_use(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return x.dtype == torch.bfloat16 and x.is_contiguous() and n <= self.max_bytes and x.numel() % 8 == 0

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        ep = self.ep
        n = x.numel()
        nbytes = n * x.element_size()
        ep.buf[:nbytes].copy_(x.view(-1).view(torch.uint8))
        out = x if out is None else out
        ep.epoch += 1
        st = stream if stream is not None else torch.cuda.current_stream(x.device)
        _native.kernels().custom_ar(out.data_ptr(), ep.buf_ptrs, ep.sig_ptrs, ep.rank, ep.world, n, ep.epoch,
                                    self.blocks, ep.err.data_ptr(), st.cuda_stream)
        return out

    def check(self) -> None:
        if int(self.ep.err.item()):
            raise RuntimeError("custom all-reduce: a peer did not arrive (barrier timeout)")


def enabled() -> bool:
    return os.environ.get("DX_CUSTOM_AR", "0") not in ("", "0")
