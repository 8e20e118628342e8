"""Sharing a KV cache with a peer process for the one-sided WRITE (round 6).

Why not hipIpcGetMemHandle: on this stack the import of a single allocation
larger than ~1 GiB never returns (`tools/ipc_probe.py`,
`profiles/r6_ipc_probe*.json`: 256 MiB and 1 GiB in < 1 ms, 2047 MiB and
2.5 GiB stuck), and a decode engine's KV cache is tens to hundreds of GiB.

So a cache that will be written by peers is allocated with the HIP virtual
memory API (`SharedKVBuffer`): ONE reserved virtual range backed by `chunk`
byte physical allocations, wrapped as a torch tensor (the engine's kernels
see an ordinary contiguous cache).  Each chunk is exportable as a dma-buf fd.
The owner serves the fds on a Unix socket (abstract namespace, SCM_RIGHTS:
the owner hands out exactly these fds, nothing else); a peer connects, gets
fresh duplicates, and maps the same chunks in the same order into a range of
its own (`RemoteMapping`).  Chunking costs nothing on the device side: the
mapping is one contiguous range on both ends.

The reference's equivalent is NIXL's memory registration + remote metadata
exchange (Patch:1296-1360); the transfer itself is agent.py / transfer.py.
"""
from __future__ import annotations

import array
import logging
import os
import socket
import struct
import threading

import torch

log = logging.getLogger("dynamo_exp_amd.disagg.kv_share")

CHUNK_BYTES = int(os.environ.get("DX_KV_SHARE_CHUNK_MB", "512")) << 20
MAX_CHUNK_BYTES = 1 << 30  # imports of single allocations above ~1 GiB were the problem: stay at or below
MAX_CHUNKS = 256  # fds the owner keeps open (and a peer receives) per cache
_MAX_FDS = 200  # per message (SCM_RIGHTS limit is 253)


def chunk_for(nbytes: int, chunk: int = CHUNK_BYTES) -> int:
    """Chunk size for an nbytes cache: `chunk`, grown so the cache takes at
    most MAX_CHUNKS fds, never above MAX_CHUNK_BYTES."""
    return min(max(chunk, -(-nbytes // MAX_CHUNKS)), MAX_CHUNK_BYTES)


def _raise_fd_limit() -> None:
    """A cache of up to MAX_CHUNKS fds per rank, and a peer mapping several:
    lift the soft open-files limit to the hard one."""
    try:
        import resource

        soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
        if soft != resource.RLIM_INFINITY and (hard == resource.RLIM_INFINITY or soft < hard):
            resource.setrlimit(resource.RLIMIT_NOFILE, (hard, hard))
    except (ImportError, ValueError, OSError) as e:
        log.warning("kv share: could not raise the open-files limit: %s", e)


class _CAI:
    """A device range as __cuda_array_interface__ (torch.as_tensor wraps it
    without taking ownership; this object keeps the owner alive)."""

    def __init__(self, ptr: int, nbytes: int, owner):
        self.owner = owner
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}


class SharedKVBuffer:
    """`nbytes` of device memory in `chunk`-byte VMM allocations, shareable
    with peer processes.  `.tensor(shape, dtype)` views it; `.address` is the
    Unix socket a peer asks for the fds on."""

    def __init__(self, nbytes: int, device: torch.device, chunk: int = CHUNK_BYTES):
        from .. import _native

        self._k = _native.kernels()
        self.device = torch.device(device)
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        _raise_fd_limit()
        self.ptr, self.total, self.chunk, self._handles = self._k.vmm_alloc(int(nbytes), chunk_for(int(nbytes), chunk),
                                                                            idx)
        self.nbytes = int(nbytes)
        self._fds = None
        self._sock = None
        self.address = None
        self._closed = False

    def tensor(self, shape, dtype: torch.dtype) -> torch.Tensor:
        n = 1
        for s in shape:
            n *= int(s)
        nb = n * torch.empty((), dtype=dtype).element_size()
        if nb > self.total:
            raise ValueError(f"view of {nb} bytes over a {self.total}-byte shared buffer")
        raw = torch.as_tensor(_CAI(self.ptr, nb, self), device=self.device)
        return raw.view(dtype).view(*shape)

    def serve(self, tag: str) -> str:
        """Start answering fd requests on an abstract Unix socket; returns
        its address (hex of the name, JSON-safe)."""
        if self.address is not None:
            return self.address
        self._fds = list(self._k.vmm_export_fds(self._handles))
        name = f"\0dx-kvshare-{os.getpid()}-{tag}".encode()
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.bind(name)
        s.listen(16)
        self._sock = s
        self.address = name.hex()
        threading.Thread(target=self._accept, daemon=True, name="kv-share").start()
        return self.address

    def _accept(self) -> None:
        while not self._closed:
            try:
                c, _ = self._sock.accept()
            except OSError:
                return
            try:
                with c:
                    c.sendall(struct.pack("<QQQ", len(self._fds), self.chunk, self.total))
                    for i in range(0, len(self._fds), _MAX_FDS):
                        part = self._fds[i:i + _MAX_FDS]
                        c.sendmsg([struct.pack("<I", len(part))],
                                  [(socket.SOL_SOCKET, socket.SCM_RIGHTS, array.array("i", part))])
            except OSError as e:  # a peer that went away: nothing to clean up here
                log.warning("kv share: peer connection failed: %s", e)

    def close(self) -> None:
        """Stop serving and free the memory (after every peer unmapped it;
        the chunks outlive this call while a peer still maps them)."""
        if self._closed:
            return
        self._closed = True
        if self._sock is not None:
            self._sock.close()
        for fd in self._fds or []:
            self._k.close_fd(fd)
        torch.cuda.synchronize(self.device)
        self._k.vmm_free(self.ptr, self.total, self._handles)


def _recv_fds(address: str, timeout: float = 30.0) -> tuple[list[int], int, int]:
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(timeout)
    s.connect(bytes.fromhex(address))
    with s:
        hdr = b""
        while len(hdr) < 24:
            b = s.recv(24 - len(hdr))
            if not b:
                raise RuntimeError("kv share: owner closed the connection")
            hdr += b
        n, chunk, total = struct.unpack("<QQQ", hdr)
        fds: list[int] = []
        while len(fds) < n:
            msg, anc, _flags, _addr = s.recvmsg(4, socket.CMSG_SPACE(_MAX_FDS * 4))
            if not msg:
                raise RuntimeError("kv share: owner closed the connection mid-transfer")
            for level, typ, data in anc:
                if level == socket.SOL_SOCKET and typ == socket.SCM_RIGHTS:
                    a = array.array("i")
                    a.frombytes(data[:len(data) - len(data) % 4])
                    fds.extend(a)
    if chunk * n != total:
        raise RuntimeError(f"kv share: {n} chunks of {chunk} bytes do not make {total}")
    return fds, chunk, total


class RemoteMapping:
    """A peer's SharedKVBuffer mapped into this process (on `device`)."""

    def __init__(self, address: str, device: torch.device):
        from .. import _native

        self._k = _native.kernels()
        _raise_fd_limit()
        fds, chunk, total = _recv_fds(address)
        dev = torch.device(device)
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        self.ptr, self.total, self._handles = self._k.vmm_import(fds, chunk, idx)
        self.chunk = chunk

    def close(self) -> None:
        if self._handles is not None:
            self._k.vmm_free(self.ptr, self.total, self._handles)
            self._handles = None
