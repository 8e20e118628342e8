"""Pinned-host KV tier (reference lib/llm/src/kv/{storage.rs,layer.rs,reuse.rs}
KV block manager v2 with device + pinned-host storage, `docs/kv_cache_manager.md:39-71`;
SURVEY §2.3 L23 / §5.8(c)).

When the device BlockPool evicts a registered (prefix-cached) block to reuse
its slot, the block is *demoted*: copied into a slot of a pinned host pool
(hipHostMalloc, mapped) and registered there under the same sequence hash.
A later prompt whose prefix misses on the device but hits on the host gets
those blocks *promoted*: fresh device blocks are filled from the host copy and
re-registered on the device (so the router sees them again).

Both copies are single launches of the block-copy kernel (K1) reading or
writing host memory through its device mapping, enqueued on the engine's
compute stream -- a demotion is therefore ordered before the forward pass
that overwrites the evicted slot, and a promotion before the forward that
reads it.  Bookkeeping (LRU over host slots, hash lookup) is a second native
BlockPool.
"""
from __future__ import annotations

import ctypes

import torch

from .. import _native, ops


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
        else:
            self.host = torch.zeros(shape, dtype=kv_cache.dtype)
            self.dev_ptr = None
        rt = _native.runtime()
        self.pool = rt.BlockPool(num_blocks, True)
        self.stats = {"demoted": 0, "promoted": 0, "demote_dropped": 0}

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

    def _copy(self, to_host: bool, gpu_ids: list[int], host_ids: list[int]) -> None:
        bb = self.block_bytes
        gpu_stride, host_stride = self.gpu_nb * bb, self.num_blocks * bb
        if to_host:
            ops.kv_copy_blocks(self.host, self.gpu, self._ids(gpu_ids), self._ids(host_ids), self.n_prefix,
                               gpu_stride, host_stride, bb, bb, bb, dst_ptr=self.dev_ptr)
        else:
            ops.kv_copy_blocks(self.gpu, self.host, self._ids(host_ids), self._ids(gpu_ids), self.n_prefix,
                               host_stride, gpu_stride, bb, bb, bb, src_ptr=self.dev_ptr)

    # ------------------------------------------------------------------ API
    def demote(self, evicted: list[tuple]) -> int:
        """evicted: [(gpu_block, seq_hash, local_hash, parent_hash|None)] whose
        device content is still intact.  Returns the number demoted."""
        evicted = [e for e in evicted if self.pool.count_prefix([e[1]]) == 0][-self.num_blocks:]
        if not evicted:
            return 0
        host_ids = self.pool.allocate(len(evicted))
        if host_ids is None:  # every host slot pinned by in-flight promotions
            self.stats["demote_dropped"] += len(evicted)
            return 0
        self._copy(True, [e[0] for e in evicted], host_ids)
        for hid, (_, seq, local, parent) in zip(host_ids, evicted):
            self.pool.register_block(hid, seq, local, parent)
        self.pool.free(host_ids)  # cached, evictable (LRU) host copies
        self.pool.drain_events()  # host-tier events are not routed
        self.stats["demoted"] += len(evicted)
        return len(evicted)

    def match(self, seq_hashes: list[int]) -> list[int]:
        """Longest host-cached prefix of seq_hashes (takes references)."""
        return list(self.pool.match_prefix(seq_hashes)) if seq_hashes else []

    def count(self, seq_hashes: list[int]) -> int:
        return self.pool.count_prefix(seq_hashes) if seq_hashes else 0

    def promote(self, host_ids: list[int], gpu_ids: list[int]) -> None:
        if host_ids:
            self._copy(False, gpu_ids, host_ids)
            self.pool.free(host_ids)
            self.stats["promoted"] += len(host_ids)

    def release(self, host_ids: list[int]) -> None:
        if host_ids:
            self.pool.free(host_ids)
