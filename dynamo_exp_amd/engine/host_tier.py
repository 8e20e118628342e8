"""Pinned-host KV tier (reference lib/llm/src/kv/{storage.rs,layer.rs,reuse.rs}
KV block manager v2 with device + pinned-host storage, `docs/kv_cache_manager.md:39-71`;
SURVEY §2.3 L23 / §5.8(c)).

When the device BlockPool evicts a registered (prefix-cached) block to reuse
its slot, the block is *demoted*: copied into a slot of a pinned host pool
(hipHostMalloc, mapped) and registered there under the same sequence hash.
A later prompt whose prefix misses on the device but hits on the host gets
those blocks *promoted*: fresh device blocks are filled from the host copy and
re-registered on the device.  Both tiers' Stored / Removed events reach the
router (KVManager merges them into one per-worker view), so host-resident
prefixes still count as overlap.

Copies run on a dedicated HIP copy stream (the reference's CopyStream,
lib/llm/src/kv/layer.rs:785-1130), single launches of the block-copy kernel
(K1) reading or writing host memory through its device mapping:

* write-ahead demotion (`write_ahead`, every engine step): the next reusable
  device blocks in eviction order are copied to the host BEFORE anything
  evicts them, behind only the compute work already enqueued; when a block is
  later evicted its host copy usually exists, so the compute stream waits for
  nothing (it waits on the copy's event only if that copy is still running);
* demotion at eviction (blocks the write-ahead did not reach): the copy is
  enqueued on the copy stream and the compute stream waits for that event
  before the forward that overwrites the slot;
* promotion: host -> device on the copy stream; the compute stream waits on
  the event before the forward that reads the blocks.

Bookkeeping (eviction order, hash lookup) is a second native BlockPool.
"""
from __future__ import annotations

import ctypes
import os

import torch

from .. import _native, ops
from ..utils import streams


def auto_host_blocks(block_bytes: int, device_blocks: int, host_fraction: float = 0.25,
                     max_device_ratio: float = 4.0) -> int:
    """Host tier size when configured as -1: up to `host_fraction` of the
    host's available RAM, at most `max_device_ratio` x the device pool (an
    MI355X node has ~3 TB of host RAM for 8 x 288 GB of HBM, so a few HBM
    pools' worth of pinned blocks per GPU is affordable), never more than the
    RAM that is actually free."""
    try:
        import psutil

        avail = psutil.virtual_memory().available
    except Exception:  # pragma: no cover
        avail = os.sysconf("SC_AVPHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
    share = int(os.environ.get("DX_HOST_KV_SHARE", "1") or 1)  # ranks sharing this host's RAM
    by_ram = int(avail * host_fraction / max(1, share)) // block_bytes
    return max(0, min(by_ram, int(device_blocks * max_device_ratio)))


class HostKVTier:
    def __init__(self, kv_cache: torch.Tensor, num_blocks: int):
        L, two, NB, H, BS, D = kv_cache.shape
        self.gpu = kv_cache
        self.num_blocks = num_blocks
        self.n_prefix = L * two
        es = kv_cache.element_size()
        self.block_bytes = H * BS * D * es
        self.gpu_nb = NB
        shape = (L, two, num_blocks, H, BS, D)
        self.on_gpu = kv_cache.is_cuda
        self._ptr = None
        if self.on_gpu:
            k = _native.kernels()
            nbytes = L * two * num_blocks * self.block_bytes
            self._ptr = k.host_alloc_pinned(nbytes)
            arr = (ctypes.c_uint8 * nbytes).from_address(self._ptr)
            self.host = torch.frombuffer(arr, dtype=torch.uint8).view(kv_cache.dtype).view(shape)
            self.dev_ptr = k.device_pointer_of_host(self._ptr)
            self.stream = streams.stream("host_tier", kv_cache.device)  # high priority: utils/streams.py
        else:
            self.host = torch.zeros(shape, dtype=kv_cache.dtype)
            self.dev_ptr = None
            self.stream = None
        rt = _native.runtime()
        self.pool = rt.BlockPool(num_blocks, True)
        self.pending: dict[int, object] = {}  # device block -> event of its in-flight write-ahead copy
        self.stats = {"demoted": 0, "promoted": 0, "demote_dropped": 0, "written_ahead": 0, "compute_waits": 0}

    def __del__(self):
        if self._ptr is not None:
            try:
                torch.cuda.synchronize()
                _native.kernels().host_free_pinned(self._ptr)
            except Exception:
                pass
            self._ptr = None

    # ------------------------------------------------------------------ copies
    def _ids(self, ids: list[int]) -> torch.Tensor:
        t = torch.tensor(ids, dtype=torch.int32)
        return t.to(self.gpu.device, non_blocking=True) if self.on_gpu else t

    def _copy(self, to_host: bool, gpu_ids: list[int], host_ids: list[int]):
        """One block-copy launch on the copy stream, after the compute work
        enqueued so far; returns its completion event (None on CPU)."""
        bb = self.block_bytes
        gpu_stride, host_stride = self.gpu_nb * bb, self.num_blocks * bb
        if self.stream is None:
            if to_host:
                ops.kv_copy_blocks(self.host, self.gpu, self._ids(gpu_ids), self._ids(host_ids), self.n_prefix,
                                   gpu_stride, host_stride, bb, bb, bb)
            else:
                ops.kv_copy_blocks(self.gpu, self.host, self._ids(host_ids), self._ids(gpu_ids), self.n_prefix,
                                   host_stride, gpu_stride, bb, bb, bb)
            return None
        self.stream.wait_stream(torch.cuda.current_stream(self.gpu.device))
        with torch.cuda.stream(self.stream):
            st = self.stream.cuda_stream
            if to_host:
                ops.kv_copy_blocks(self.host, self.gpu, self._ids(gpu_ids), self._ids(host_ids), self.n_prefix,
                                   gpu_stride, host_stride, bb, bb, bb, dst_ptr=self.dev_ptr, stream=st)
            else:
                ops.kv_copy_blocks(self.gpu, self.host, self._ids(host_ids), self._ids(gpu_ids), self.n_prefix,
                                   host_stride, gpu_stride, bb, bb, bb, src_ptr=self.dev_ptr, stream=st)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return ev

    def _compute_waits(self, ev) -> None:
        if ev is not None and not ev.query():
            torch.cuda.current_stream(self.gpu.device).wait_event(ev)
            self.stats["compute_waits"] += 1

    def _store(self, entries: list[tuple]) -> tuple[list[int], object] | None:
        """Copy device blocks [(gpu_block, seq, local, parent)] to fresh host
        slots and register them there; returns (host ids, event)."""
        host_ids = self.pool.allocate(len(entries))
        if host_ids is None:  # every host slot pinned by in-flight promotions
            self.stats["demote_dropped"] += len(entries)
            return None
        ev = self._copy(True, [e[0] for e in entries], host_ids)
        for hid, (_, seq, local, parent) in zip(host_ids, entries):
            self.pool.register_block(hid, seq, local, parent)
        self.pool.free(host_ids)  # cached, evictable host copies
        return host_ids, ev

    # ------------------------------------------------------------------ API
    def write_ahead(self, device_pool, n: int) -> int:
        """Copy up to n of the device pool's next-to-be-evicted blocks that have
        no host copy yet (no compute-stream dependency)."""
        entries = []
        for b in device_pool.lru_candidates(n):
            info = device_pool.block_info(b)
            if info is None or b in self.pending or self.pool.count_prefix([info[0]]):
                continue
            entries.append((b, info[0], info[1], info[2]))
        if not entries:
            return 0
        res = self._store(entries)
        if res is None:
            return 0
        for e in entries:
            self.pending[e[0]] = res[1]
        self.stats["written_ahead"] += len(entries)
        return len(entries)

    def demote(self, evicted: list[tuple]) -> int:
        """evicted: [(gpu_block, seq_hash, local_hash, parent_hash|None)] whose
        device content is still intact; the compute stream must not overwrite
        them before their copy read them.  Returns the number copied now."""
        for e in evicted:  # written ahead: wait only if that copy still runs
            self._compute_waits(self.pending.pop(e[0], None))
        todo = [e for e in evicted if self.pool.count_prefix([e[1]]) == 0][-self.num_blocks:]
        if not todo:
            return 0
        res = self._store(todo)
        if res is None:
            return 0
        self._compute_waits(res[1])
        self.stats["demoted"] += len(todo)
        return len(todo)

    def forget_pending(self) -> None:
        """Write-ahead copies whose device blocks were re-referenced or reset:
        drop the events that finished (the host copies stay valid)."""
        for b in [b for b, ev in self.pending.items() if ev is None or ev.query()]:
            del self.pending[b]

    def match(self, seq_hashes: list[int]) -> list[int]:
        """Longest host-cached prefix of seq_hashes (takes references)."""
        return list(self.pool.match_prefix(seq_hashes)) if seq_hashes else []

    def count(self, seq_hashes: list[int]) -> int:
        return self.pool.count_prefix(seq_hashes) if seq_hashes else 0

    def promote(self, host_ids: list[int], gpu_ids: list[int]) -> None:
        if host_ids:
            ev = self._copy(False, gpu_ids, host_ids)
            if ev is not None:  # the forward reading these blocks runs after the copy
                torch.cuda.current_stream(self.gpu.device).wait_event(ev)
            self.pool.free(host_ids)
            self.stats["promoted"] += len(host_ids)

    def release(self, host_ids: list[int]) -> None:
        if host_ids:
            self.pool.free(host_ids)
