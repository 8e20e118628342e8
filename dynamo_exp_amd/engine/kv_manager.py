"""Per-request paged-KV bookkeeping on top of the native :class:`BlockPool`.

* prompt admission: longest cached prefix (sequence-hash lookup), then fresh
  blocks for the rest; at least one prompt token is always recomputed so the
  first output token has logits;
* incremental registration of blocks as they fill (prompt *and* generated
  tokens), producing the router's KV events (Stored / Removed) with the
  reference's hashing (see :mod:`dynamo_exp_amd.kv.hashing`);
* decode growth, free/release (a request's `cache_priority` ranks its blocks
  in the eviction order: lowest priority first, then oldest release --
  reference reuse.rs PriorityKey);
* with a pinned-host tier: one per-worker view of both tiers for the router
  (a hash is Stored while either tier holds it, Removed when neither does)
  and write-ahead demotion of the next blocks to be evicted.
"""
from __future__ import annotations

from typing import Callable

from .. import _native
from ..kv import hashing
from .request import Request


class KVEvent:
    __slots__ = ("kind", "seq_hash", "local_hash", "parent_hash", "medium")

    def __init__(self, kind: str, seq_hash: int, local_hash: int, parent_hash: int | None, medium: str = "device"):
        self.kind, self.seq_hash, self.local_hash, self.parent_hash = kind, seq_hash, local_hash, parent_hash
        self.medium = medium  # tier whose change caused the event: "device" | "host"

    def __repr__(self):
        return f"KVEvent({self.kind}, {self.seq_hash:x})"


class KVManager:
    def __init__(self, num_blocks: int, block_size: int, enable_prefix_caching: bool = True,
                 event_sink: Callable[[list[KVEvent]], None] | None = None, host_tier=None):
        rt = _native.runtime()
        if rt is None:
            raise RuntimeError("dynamo_exp_amd._C_runtime is required (BlockPool)")
        self.pool = rt.BlockPool(num_blocks, enable_prefix_caching)
        self.host = host_tier if enable_prefix_caching else None
        if self.host is not None:
            self.pool.set_track_evictions(True)
        self.host_hit_tokens = 0
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.caching = enable_prefix_caching
        self.event_sink = event_sink
        self.prefix_queries = 0
        self.prefix_hit_tokens = 0
        self.prefix_query_tokens = 0
        self._tiers: dict[int, int] = {}  # seq hash -> tier bits (1 device, 2 host), host tier only
        # write-ahead demotion keeps this many upcoming evictions copied to the host
        self.write_ahead_blocks = max(8, num_blocks // 64)

    # ------------------------------------------------------------- capacity
    def num_free(self) -> int:
        return self.pool.num_free()

    def usage(self) -> float:
        return 1.0 - self.pool.num_free() / max(1, self.num_blocks)

    def blocks_needed(self, n_tokens: int) -> int:
        return (n_tokens + self.block_size - 1) // self.block_size

    # ------------------------------------------------------------- prompt
    def prefix_hit_tokens_for(self, prompt: list[int]) -> int:
        if not self.caching:
            return 0
        _, seq = hashing.block_and_sequence_hashes(prompt, self.block_size)
        n = self.pool.count_prefix(seq)
        if self.host is not None:
            n += self.host.count(seq[n:])
        return n * self.block_size

    def _allocate(self, n: int):
        """Device blocks; registered blocks evicted to make room are demoted
        to the host tier first (copy enqueued before any overwrite)."""
        new = self.pool.allocate(n)
        if self.host is not None:
            ev = self.pool.drain_evicted()
            if ev:
                self.host.demote(ev)
        return new

    def allocate_prompt(self, req: Request, reserve_tokens: int = 1, use_cache: bool = True) -> bool:
        """Admit `req`: reuse cached prefix blocks and allocate the rest of the
        prompt plus `reserve_tokens` slots.  Returns False if KV is exhausted."""
        bs = self.block_size
        P = len(req.prompt)
        hits: list[int] = []
        host_hits: list[int] = []
        bh, sh = [], []
        if self.caching and use_cache:
            hp = req.hash_prompt if req.hash_prompt is not None else req.prompt
            bh, sh = hashing.block_and_sequence_hashes(hp, bs)
            max_hit_blocks = (P - 1) // bs  # keep >= 1 token to compute
            hits = list(self.pool.match_prefix(sh[:max_hit_blocks]))
            if self.host is not None:
                host_hits = self.host.match(sh[len(hits):max_hit_blocks])
        need = self.blocks_needed(P + reserve_tokens) - len(hits)
        new = self._allocate(max(0, need))
        if new is None:
            if hits:
                self.pool.free(hits)
            if host_hits:
                self.host.release(host_hits)
            return False
        new = list(new)
        if host_hits:
            # promote: fill fresh device blocks from the host copies, re-register
            k0, nh = len(hits), len(host_hits)
            self.host.promote(host_hits, new[:nh])
            for i in range(nh):
                parent = sh[k0 + i - 1] if k0 + i > 0 else None
                self.pool.register_block(new[i], sh[k0 + i], bh[k0 + i], parent)
            self.host_hit_tokens += nh * bs
            self._flush_events()
        n_cached = len(hits) + len(host_hits)
        req.block_ids = hits + new
        req.num_computed = n_cached * bs
        req.num_prefix_hit = req.num_computed
        req.block_hashes = bh[:n_cached]
        req.seq_hashes = sh[:n_cached]
        self.prefix_queries += 1
        self.prefix_hit_tokens += req.num_prefix_hit
        self.prefix_query_tokens += P
        return True

    def allocate_for_remote(self, req: Request, reserve_tokens: int = 1) -> bool:
        """Decode side of disaggregation: blocks for prompt (+ first token) that
        a prefill worker will fill.  Cached prefix blocks are reused and the
        remote worker is told which are already computed."""
        return self.allocate_prompt(req, reserve_tokens=reserve_tokens)

    # ------------------------------------------------------------- decode growth
    def ensure_slots(self, req: Request, total_tokens: int) -> bool:
        need = self.blocks_needed(total_tokens) - len(req.block_ids)
        if need <= 0:
            return True
        new = self._allocate(need)
        if new is None:
            return False
        req.block_ids.extend(new)
        return True

    # ------------------------------------------------------------- registration
    def register_filled(self, req: Request) -> None:
        """Register every block of `req` fully covered by computed tokens."""
        if not self.caching:
            return
        bs = self.block_size
        n_full = req.num_computed // bs
        done = len(req.seq_hashes)
        if n_full <= done:
            return
        toks = req.hash_tokens()
        new_bh = hashing.block_hashes(toks[done * bs: n_full * bs], bs)
        parent = req.seq_hashes[-1] if req.seq_hashes else None
        new_sh = hashing.chain_hashes(new_bh, parent)
        for i, (b, s) in enumerate(zip(new_bh, new_sh)):
            idx = done + i
            p = req.seq_hashes[-1] if req.seq_hashes else None
            self.pool.register_block(req.block_ids[idx], s, b, p)
            req.block_hashes.append(b)
            req.seq_hashes.append(s)
        self._flush_events()

    def free(self, req: Request) -> None:
        if req.block_ids:
            self.pool.free(req.block_ids, int(getattr(req.params, "cache_priority", 0) or 0))
            req.block_ids = []
        self._flush_events()

    def set_priority(self, seq_hashes: list[int], priority: int) -> int:
        """Re-rank cached blocks (reference reuse.rs update_block); returns how many were found."""
        return sum(bool(self.pool.set_priority(h, priority)) for h in seq_hashes)

    def maintain(self) -> None:
        """Once per engine step: keep the next evictions' host copies ahead."""
        if self.host is not None:
            self.host.forget_pending()
            if self.pool.num_free() < 4 * self.write_ahead_blocks:
                self.host.write_ahead(self.pool, self.write_ahead_blocks)
            self._flush_events()

    def reset_prefix_cache(self) -> int:
        """Forget every cached block that is not in use, on both tiers
        (Removed events for all of them)."""
        n = self.pool.reset_cache()
        if self.host is not None:
            self.pool.drain_evicted()  # a reset forgets, it does not demote
            n += self.host.pool.reset_cache()
            self.host.pending.clear()  # in-flight write-aheads only fill host slots that are now free
        self._flush_events()
        return n

    def _flush_events(self) -> None:
        ev = self.pool.drain_events()
        if self.host is None:
            if ev and self.event_sink is not None:
                self.event_sink([KVEvent("stored" if k == 0 else "removed", s, l, p) for (k, s, l, p) in ev])
            return
        hev = self.host.pool.drain_events()
        if not ev and not hev:
            return
        out = []
        # host first: a demotion (device Removed + host Stored of one hash in
        # one flush) then leaves the router's view unchanged
        for bit, medium, evs in ((2, "host", hev), (1, "device", ev)):
            for k, sh, lh, ph in evs:
                before = self._tiers.get(sh, 0)
                after = before | bit if k == 0 else before & ~bit
                if after:
                    self._tiers[sh] = after
                else:
                    self._tiers.pop(sh, None)
                if not before and after:
                    out.append(KVEvent("stored", sh, lh, ph, medium))
                elif before and not after:
                    out.append(KVEvent("removed", sh, lh, ph, medium))
        if out and self.event_sink is not None:
            self.event_sink(out)

    def hit_rate(self) -> float:
        return self.prefix_hit_tokens / self.prefix_query_tokens if self.prefix_query_tokens else 0.0
