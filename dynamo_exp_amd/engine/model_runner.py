"""Model runner: paged KV allocation, batch tensor preparation, hipGraph
decode capture and sampling on the GPU.

Pure decode steps are captured into HIP graphs (torch.cuda.graph on ROCm)
per batch-size bucket; every per-step input lives in a static device buffer
that is refreshed with one async H2D copy from a pinned staging buffer before
the replay, so a decode step costs one graph launch plus one small copy.
Prefill and mixed (prompt chunks + decode rows) steps run eagerly: one token
stream [prefill tokens | decode tokens] through the GEMMs, prefill attention
on the first part and split-K decode attention on the rest.
"""
from __future__ import annotations

import bisect
import collections
import gc
import math
import os
import zlib
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops
from ..models.llama import AttnMeta, LlamaForCausalLM
from .request import Request

# device-time accounting with CUDA events around each launch (DX_GPU_TIMING=0: off)
_GPU_TIMING = os.environ.get("DX_GPU_TIMING", "1") != "0"

DEFAULT_GRAPH_SIZES = [1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256]


@dataclass
class RunnerConfig:
    block_size: int = 64
    num_gpu_blocks: int | None = None  # None -> derived from gpu_memory_utilization
    gpu_memory_utilization: float = 0.90
    max_model_len: int = 8192
    max_num_seqs: int = 256
    use_cuda_graph: bool = True
    graph_sizes: tuple = tuple(DEFAULT_GRAPH_SIZES)
    kv_dtype: torch.dtype = torch.bfloat16
    kv_shared: bool = False  # allocate the cache shareable with peer processes (disagg/kv_share.py)


@dataclass
class Launched:
    """A batch whose forward is enqueued and whose sampled tokens have not been
    read back (asynchronous scheduling): device results, their pinned-host
    copies in flight, and where each request's token sits."""

    tok: torch.Tensor
    lp: torch.Tensor
    rows: dict = field(default_factory=dict)  # request id -> row of tok / lp
    host: tuple | None = None  # pinned (tok, lp) destinations of the async D2H
    event: object = None
    t0: float = 0.0
    prefill: bool = False


class ModelRunner:
    def __init__(self, model: LlamaForCausalLM, cfg: RunnerConfig):
        self.model = model
        self.cfg = cfg
        self.device = model.device
        self.is_gpu = self.device.type == "cuda"
        mc = model.cfg
        self.block_size = cfg.block_size
        self.max_blocks_per_seq = math.ceil(cfg.max_model_len / cfg.block_size)
        # fp8 KV: the prefill attention reads a bf16 dequant scratch of the
        # prefill sequences' live blocks, packed and capped at this many blocks
        # per layer (batches beyond it run attention in sequence groups);
        # reserved out of the KV budget (it used to grow unbounded)
        self.kv_fp8 = cfg.kv_dtype == torch.float8_e4m3fn
        self.fp8_scratch_cap = max(2 * self.max_blocks_per_seq, 256) if self.kv_fp8 else 0
        self.num_blocks = cfg.num_gpu_blocks or self._auto_blocks()
        L = mc.num_hidden_layers
        shape = (L, 2, self.num_blocks, model.n_kv, cfg.block_size, model.head_dim)
        self.kv_share = None
        if cfg.kv_shared and self.is_gpu:
            from ..disagg.kv_share import SharedKVBuffer

            nbytes = math.prod(shape) * torch.empty((), dtype=cfg.kv_dtype).element_size()
            self.kv_share = SharedKVBuffer(nbytes, self.device)
            self.kv_cache = self.kv_share.tensor(shape, cfg.kv_dtype)
            self.kv_cache.zero_()
        else:
            self.kv_cache = torch.zeros(shape, dtype=cfg.kv_dtype, device=self.device)
        self.kv_caches = [(self.kv_cache[i, 0], self.kv_cache[i, 1]) for i in range(L)]
        self.graphs: dict[int, tuple] = {}
        self.graphs_sharded: dict[int, object] = {}  # TP > 1: vocab-sharded sampler variant
        self._res_tok = self._res_lp = None  # multi-step decode result buffers
        self.graph_pool = None
        self._static = None
        self.vocab = mc.vocab_size
        self.step_times: list[float] = []
        self._pinned_ring: list[tuple] = []  # async read-back buffers (pinned host)
        self._ring_i = 0
        # *_gpu: device time of the batches (CUDA events around each launch,
        # harvested once they completed; on CPU the launch is the execution);
        # *_wait: host time blocked reading results back
        self.timing = {"prefill_prep": 0.0, "prefill_gpu": 0.0, "decode_prep": 0.0, "decode_gpu": 0.0,
                       "prefill_wait": 0.0, "decode_wait": 0.0,
                       "prefill_tokens": 0, "prefill_steps": 0, "decode_steps": 0, "decode_seqs": 0}
        self._gpu_events: collections.deque = collections.deque()  # (kind, start, end) not yet harvested

    # ------------------------------------------------------------------ memory
    def _auto_blocks(self) -> int:
        mc = self.model.cfg
        per_block = (mc.num_hidden_layers * 2 * self.model.n_kv * self.cfg.block_size * self.model.head_dim *
                     torch.empty((), dtype=self.cfg.kv_dtype).element_size())
        if not self.is_gpu:
            return max(64, (256 << 20) // per_block)
        free, total = torch.cuda.mem_get_info(self.device)
        budget = total * self.cfg.gpu_memory_utilization - (total - free)
        # activations / graphs / logits headroom
        budget -= 6 << 30
        # fp8 prefill dequant scratch (bf16 K + V, one layer at a time)
        budget -= self.fp8_scratch_cap * 2 * self.model.n_kv * self.cfg.block_size * self.model.head_dim * 2
        n = int(budget // per_block)
        if n <= 0:
            raise RuntimeError("not enough GPU memory for the KV cache")
        return n

    @property
    def kv_bytes(self) -> int:
        return self.kv_cache.numel() * self.kv_cache.element_size()

    def block_bytes_per_layer(self) -> int:
        return self.model.n_kv * self.block_size * self.model.head_dim * self.kv_cache.element_size()

    # ------------------------------------------------------------------ prep
    def _to_dev(self, arr: np.ndarray, dtype) -> torch.Tensor:
        t = torch.from_numpy(arr)
        if self.is_gpu:
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t.to(dtype) if t.dtype != dtype else t

    def _block_table(self, reqs: list[Request], width: int | None = None) -> np.ndarray:
        width = width or max(1, max(len(r.block_ids) for r in reqs))
        bt = np.zeros((len(reqs), width), dtype=np.int32)
        for i, r in enumerate(reqs):
            n = min(len(r.block_ids), width)
            bt[i, :n] = r.block_ids[:n]
        return bt

    def prepare_prefill(self, reqs: list[Request], num_new: list[int], sample: list[bool] | None = None,
                        decode: list[Request] | None = None):
        """Token stream + metadata for prompt chunks `reqs` (num_new tokens
        each) followed by one decode token per request in `decode`."""
        bs = self.block_size
        decode = decode or []
        sample = sample if sample is not None else [True] * len(reqs)
        ids, pos, slots = [], [], []
        cu = [0]
        ctx = []
        mm_rows, mm_parts = [], []
        for r, n in zip(reqs, num_new):
            start = r.num_computed
            toks = r.prompt[start:start + n]
            if r.mm_positions:  # image embeddings landing in this chunk
                i0 = bisect.bisect_left(r.mm_positions, start)
                i1 = bisect.bisect_left(r.mm_positions, start + n)
                if i1 > i0:
                    mm_rows.extend(len(ids) + p - start for p in r.mm_positions[i0:i1])
                    mm_parts.append(r.mm_embeds[i0:i1])
            ids.extend(toks)
            p = np.arange(start, start + n, dtype=np.int64)
            pos.append(p)
            bt = np.asarray(r.block_ids, dtype=np.int64)
            slots.append(bt[p // bs] * bs + p % bs)
            cu.append(cu[-1] + n)
            ctx.append(start + n)
        Tp = cu[-1]
        rows = [c - 1 for c, s_ in zip(cu[1:], sample) if s_]
        dmeta = None
        if decode:
            B = len(decode)
            d_ids, d_pos, d_slots, d_ctx = self._decode_host_inputs(decode, B)
            ids.extend(d_ids.tolist())
            pos.append(d_pos)
            slots.append(d_slots)
            rows.extend(range(Tp, Tp + B))
            dmeta = AttnMeta(is_prefill=False, positions=None, slot_mapping=None,
                             block_tables=self._to_dev(self._block_table(decode), torch.int32),
                             ctx_lens=self._to_dev(d_ctx, torch.int32), n_parts=self._n_parts(B))
            if self.is_gpu:
                dmeta.workspace = ops.decode_workspace(B, self.model.n_q, self.model.head_dim, dmeta.n_parts,
                                                       self.device)
        pos = np.concatenate(pos)
        slots = np.concatenate(slots)
        mc = self.model
        work = ops.prefill_work_list(num_new, ctx, mc.n_q, mc.n_kv) if reqs else []
        meta = AttnMeta(
            is_prefill=True,
            positions=self._to_dev(pos, torch.int64),
            slot_mapping=self._to_dev(slots, torch.int64),
            block_tables=self._to_dev(self._block_table(reqs), torch.int32) if reqs else None,
            ctx_lens=self._to_dev(np.asarray(ctx, dtype=np.int32), torch.int32) if reqs else None,
            cu_seqlens_q=self._to_dev(np.asarray(cu, dtype=np.int32), torch.int32),
            work=self._to_dev(np.asarray(work, dtype=np.int32), torch.int32) if reqs else None,
            logits_idx=self._to_dev(np.asarray(rows, dtype=np.int64), torch.int64),
            num_prefill_tokens=Tp,
            decode=dmeta,
        )
        if reqs and self.kv_fp8 and self.is_gpu:
            self._plan_fp8_scratch(meta, reqs, num_new, ctx, cu)
        if mm_rows:
            meta.mm_rows = self._to_dev(np.asarray(mm_rows, dtype=np.int64), torch.int64)
            meta.mm_embeds = torch.cat(mm_parts) if len(mm_parts) > 1 else mm_parts[0]
        return self._to_dev(np.asarray(ids, dtype=np.int64), torch.int64), meta

    def _plan_fp8_scratch(self, meta, reqs, num_new, ctx, cu) -> None:
        """Packed (and, past the cap, sequence-grouped) dequant scratch of an
        fp8 cache's prefill rows (ops.fp8_scratch_plan)."""
        width = meta.block_tables.shape[1]
        groups = ops.fp8_scratch_plan(ctx, self.block_size, width, self.fp8_scratch_cap)
        if len(groups) == 1:
            meta.fp8_scratch = (self._to_dev(groups[0][3], torch.int32), groups[0][2])
            return
        mc = self.model
        meta.fp8_groups = []
        for s0, s1, nb, tab in groups:
            t0, t1 = cu[s0], cu[s1]
            cu_g = np.asarray([c - t0 for c in cu[s0:s1 + 1]], dtype=np.int32)
            work = ops.prefill_work_list(num_new[s0:s1], ctx[s0:s1], mc.n_q, mc.n_kv)
            meta.fp8_groups.append((t0, t1, s0, s1, self._to_dev(cu_g, torch.int32),
                                    self._to_dev(np.asarray(work, dtype=np.int32), torch.int32),
                                    self._to_dev(tab, torch.int32), nb))

    def _decode_host_inputs(self, reqs: list[Request], B: int):
        bs = self.block_size
        ids = np.zeros(B, dtype=np.int64)
        pos = np.zeros(B, dtype=np.int64)
        slots = np.full(B, -1, dtype=np.int64)
        ctx = np.zeros(B, dtype=np.int32)
        for i, r in enumerate(reqs):
            p = r.num_tokens - 1
            ids[i] = r.output[-1] if r.output else r.prompt[-1]
            pos[i] = p
            slots[i] = r.block_ids[p // bs] * bs + p % bs
            ctx[i] = p + 1
        return ids, pos, slots, ctx

    def _sampling_host(self, reqs: list[Request], B: int):
        temp = np.zeros(B, dtype=np.float32)
        topk = np.zeros(B, dtype=np.int32)
        topp = np.ones(B, dtype=np.float32)
        minp = np.zeros(B, dtype=np.float32)
        seeds = np.zeros(B, dtype=np.int64)
        offs = np.zeros(B, dtype=np.int64)
        for i, r in enumerate(reqs):
            p = r.params
            temp[i] = p.temperature
            topk[i] = p.top_k
            topp[i] = p.top_p
            minp[i] = p.min_p
            seeds[i] = p.seed if p.seed is not None else (zlib.crc32(r.request_id.encode()) * 2654435761) & 0x7FFFFFFFFFFF
            offs[i] = r.sample_offset
        return temp, topk, topp, minp, seeds, offs

    # ------------------------------------------------------------------ execute
    @torch.inference_mode()
    def execute(self, batch):
        """Run one scheduler Batch; returns (tokens, logprobs) for
        `batch.sampled` in order (synchronous: waits for the GPU)."""
        return self.fetch(self.launch(batch, None, readback=False))

    @torch.inference_mode()
    def launch(self, batch, prev: Launched | None, readback: bool = True) -> Launched:
        """Enqueue one batch.  Decode rows whose input token is still a
        placeholder (sampled by `prev`, in flight) take it from prev's device
        result.  readback: start the pinned-host copy of the sampled tokens
        right behind the forward (fetch waits only for that)."""
        t0 = time.perf_counter()
        tm = self.timing
        ev0 = None
        if self.is_gpu and _GPU_TIMING:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        npre = batch.n_prefill
        if npre:
            reqs = batch.requests[:npre]
            decode = batch.requests[npre:]
            ids, meta = self.prepare_prefill(reqs, batch.num_new, batch.sample, decode)
            patch = self._placeholder_rows(decode, meta.num_prefill_tokens, prev)
            if patch:
                self._patch_ids(ids, patch, prev)
            sampled = batch.sampled
            if sampled:
                hidden = self.model.forward(ids, meta, self.kv_caches)
                tok, lp = self._sample_hidden(hidden, sampled)
            else:  # only partial chunks: no logits needed
                meta.logits_idx = meta.logits_idx[:0]
                self.model.forward(ids, meta, self.kv_caches)
                tok = lp = torch.empty(0)
            tm["prefill_prep"] += time.perf_counter() - t0
            tm["prefill_tokens"] += sum(batch.num_new)
            tm["prefill_steps"] += 1
            tm["decode_seqs"] += len(decode)
        else:
            reqs = batch.requests
            B = len(reqs)
            patch = self._placeholder_rows(reqs, 0, prev)
            gb = self._graph_bucket(B)
            if gb is not None and not any(r.params.needs_penalties for r in reqs):
                tok, lp = self._run_graph(gb, reqs, patch, prev)
            else:
                tok, lp = self._run_decode_eager(reqs, patch, prev)
            tm["decode_prep"] += time.perf_counter() - t0
            tm["decode_steps"] += 1
            tm["decode_seqs"] += B
        out = Launched(tok, lp, {r.request_id: i for i, r in enumerate(batch.sampled)}, t0=t0, prefill=bool(npre))
        kind = "prefill" if npre else "decode"
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self._gpu_events.append((kind, ev0, ev1))
        elif not self.is_gpu:
            tm[f"{kind}_gpu"] += time.perf_counter() - t0
        if readback and self.is_gpu and tok.numel():
            out.host = self._readback(tok, lp)
            out.event = torch.cuda.Event()
            out.event.record()
        return out

    def fetch(self, h: Launched) -> tuple[list[int], list[float]]:
        """Host values of a launched batch's tokens (waits for them)."""
        t1 = time.perf_counter()
        if h.host is not None:
            h.event.synchronize()
            n = h.tok.numel()
            out_t = h.host[0][:n].tolist()
            out_l = h.host[1][:n].tolist()
        else:
            out_t = h.tok.tolist()
            out_l = h.lp.tolist()
        t2 = time.perf_counter()
        self.timing["prefill_wait" if h.prefill else "decode_wait"] += t2 - t1
        self.step_times.append(t2 - h.t0)
        self.harvest_gpu_time()
        return out_t, out_l

    def harvest_gpu_time(self) -> None:
        """Add the device time of every completed launch to *_gpu."""
        q = self._gpu_events
        while q and q[0][2].query():
            kind, a, b = q.popleft()
            self.timing[f"{kind}_gpu"] += a.elapsed_time(b) / 1e3

    def _readback(self, tok: torch.Tensor, lp: torch.Tensor) -> tuple:
        """Non-blocking D2H into a ring of pinned buffers (a batch is fetched
        before the ring wraps: one batch in flight at a time)."""
        n = tok.numel()
        if not self._pinned_ring or self._pinned_ring[0][0].numel() < n:
            cap = max(n, self.cfg.max_num_seqs + 256)
            self._pinned_ring = [(torch.empty(cap, dtype=torch.int64).pin_memory(),
                                  torch.empty(cap, dtype=torch.float32).pin_memory()) for _ in range(3)]
        ht, hl = self._pinned_ring[self._ring_i % len(self._pinned_ring)]
        self._ring_i += 1
        ht[:n].copy_(tok.to(torch.int64), non_blocking=True)
        hl[:n].copy_(lp.to(torch.float32), non_blocking=True)
        return ht, hl

    @staticmethod
    def _placeholder_rows(reqs: list[Request], row0: int, prev: Launched | None) -> list[tuple[int, int]]:
        """(token-stream row, prev result row) of decode rows whose input
        token is a placeholder sampled by the batch in flight."""
        if prev is None:
            return []
        out = []
        for i, r in enumerate(reqs):
            if r.pending:
                out.append((row0 + i, prev.rows[r.request_id]))
        return out

    def _patch_ids(self, ids: torch.Tensor, patch: list[tuple[int, int]], prev: Launched) -> None:
        dst = self._to_dev(np.asarray([p[0] for p in patch], dtype=np.int64), torch.int64)
        src = self._to_dev(np.asarray([p[1] for p in patch], dtype=np.int64), torch.int64)
        ids.index_copy_(0, dst, prev.tok.to(ids.device).index_select(0, src).to(ids.dtype))

    def _sharded_ok(self, reqs: list[Request]) -> bool:
        """TP > 1: rows that can be sampled per vocab shard (greedy or plain
        temperature); top-k / top-p / min-p / penalties need the full logits."""
        return all(r.params.top_k <= 0 and r.params.top_p >= 1.0 and r.params.min_p <= 0.0
                   and not r.params.needs_penalties for r in reqs)

    def _sample_hidden(self, hidden, reqs):
        if self.model.tp.size > 1 and self._sharded_ok(reqs):
            temp, _, _, _, seeds, offs = self._sampling_host(reqs, len(reqs))
            return self.model.sample_sharded(hidden, self._to_dev(temp, torch.float32),
                                             self._to_dev(seeds, torch.int64), self._to_dev(offs, torch.int64))
        return self._sample(self.model.compute_logits(hidden), reqs)

    def _sample(self, logits, reqs):
        B = len(reqs)
        if any(r.params.needs_penalties for r in reqs):
            ops.apply_penalties(logits, [r.output for r in reqs], [r.prompt for r in reqs],
                                [r.params.repetition_penalty for r in reqs], [r.params.frequency_penalty for r in reqs],
                                [r.params.presence_penalty for r in reqs])
        host = self._sampling_host(reqs, B)
        greedy = all(r.params.temperature <= 0 for r in reqs)
        if greedy:
            t = self._to_dev(host[0], torch.float32)
            return ops.sample(logits, t)
        dmap = {np.dtype(np.float32): torch.float32, np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64}
        d = [self._to_dev(h, dmap[h.dtype]) for h in host]
        return ops.sample(logits, *d)

    def _run_decode_eager(self, reqs, patch=None, prev=None):
        B = len(reqs)
        ids, pos, slots, ctx = self._decode_host_inputs(reqs, B)
        meta = AttnMeta(
            is_prefill=False,
            positions=self._to_dev(pos, torch.int64),
            slot_mapping=self._to_dev(slots, torch.int64),
            block_tables=self._to_dev(self._block_table(reqs), torch.int32),
            ctx_lens=self._to_dev(ctx, torch.int32),
            n_parts=self._n_parts(B),
        )
        if self.is_gpu:
            meta.workspace = ops.decode_workspace(B, self.model.n_q, self.model.head_dim, meta.n_parts, self.device)
        ids_t = self._to_dev(ids, torch.int64)
        if patch:
            self._patch_ids(ids_t, patch, prev)
        hidden = self.model.forward(ids_t, meta, self.kv_caches)
        return self._sample_hidden(hidden, reqs)

    # ------------------------------------------------------------------ graphs
    def _n_parts(self, B: int) -> int:
        return ops.decode_num_parts(B, self.model.n_kv, self.cfg.max_model_len)

    def _graph_workspace(self, B: int):
        P, Hq, D = self._n_parts(B), self.model.n_q, self.model.head_dim
        return (self._workspace[0][:B * Hq * P * D].view(B, Hq, P, D),
                self._workspace[1][:B * Hq * P * 2].view(B, Hq, P, 2))

    def _graph_bucket(self, B: int) -> int | None:
        if not (self.is_gpu and self.cfg.use_cuda_graph):
            return None
        for s in self.cfg.graph_sizes:
            if s >= B and s in self.graphs:
                return s
        return None

    def _alloc_static(self):
        maxB = max(self.cfg.graph_sizes)
        dev = self.device
        mb = self.max_blocks_per_seq
        # one pinned host staging buffer + one device buffer, sliced per field (single H2D per step)
        self._layout = [("ids", torch.int64, maxB), ("pos", torch.int64, maxB), ("slots", torch.int64, maxB),
                        ("seeds", torch.int64, maxB), ("offs", torch.int64, maxB), ("ctx", torch.int32, maxB),
                        ("topk", torch.int32, maxB), ("bt", torch.int32, maxB * mb), ("temp", torch.float32, maxB),
                        ("topp", torch.float32, maxB), ("minp", torch.float32, maxB)]
        nbytes = 0
        self._offsets = {}
        for name, dt, n in self._layout:
            sz = n * torch.tensor([], dtype=dt).element_size()
            self._offsets[name] = (nbytes, dt, n)
            nbytes += (sz + 255) // 256 * 256
        self._dev_buf = torch.zeros(nbytes, dtype=torch.uint8, device=dev)

        def view(buf, name):
            off, dt, n = self._offsets[name]
            return buf[off:off + n * torch.tensor([], dtype=dt).element_size()].view(dt)

        def views(buf):
            v = {name: view(buf, name) for name, _, _ in self._layout}
            v["bt"] = v["bt"].view(maxB, mb)
            return v

        # Two pinned host staging buffers used in turn, each with the event of
        # its last H2D: under asynchronous scheduling step t+1's inputs are
        # written while step t's non-blocking H2D may still be queued, so a
        # single buffer could be overwritten before the DMA read it.  A buffer
        # is rewritten only once its previous copy completed (the wait is a
        # no-op in practice: two steps separate the uses).
        self._host_bufs = [torch.zeros(nbytes, dtype=torch.uint8).pin_memory() for _ in range(2)]
        self._hvs = [views(b) for b in self._host_bufs]
        self._h2d_done: list = [None, None]
        self._hb = 0
        self._host_buf, self._hv = self._host_bufs[0], self._hvs[0]
        self._dv = views(self._dev_buf)
        self._out_tok = torch.zeros(maxB, dtype=torch.int64, device=dev)
        self._out_lp = torch.zeros(maxB, dtype=torch.float32, device=dev)
        # one flat decode-attention workspace, viewed per bucket as [B, Hq, P(B), ...]
        ws = max(B * self._n_parts(B) for B in self.cfg.graph_sizes)
        self._workspace = (torch.empty(ws * self.model.n_q * self.model.head_dim, dtype=torch.float32, device=dev),
                           torch.empty(ws * self.model.n_q * 2, dtype=torch.float32, device=dev))
        self._static = True

    def _graph_forward(self, B: int, full: bool = True):
        """One decode step for graph capture.  `full=False` (TP > 1 only):
        the vocab-sharded sampler (no logits gather) for greedy/temperature
        batches; `full=True`: full logits + the top-k/top-p/min-p sampler."""
        dv = self._dv
        meta = AttnMeta(
            is_prefill=False,
            positions=dv["pos"][:B],
            slot_mapping=dv["slots"][:B],
            block_tables=dv["bt"][:B],
            ctx_lens=dv["ctx"][:B],
            n_parts=self._n_parts(B),
            workspace=self._graph_workspace(B),
        )
        hidden = self.model.forward(dv["ids"][:B], meta, self.kv_caches)
        if not full:
            self.model.sample_sharded(hidden, dv["temp"][:B], dv["seeds"][:B], dv["offs"][:B],
                                      out_tokens=self._out_tok[:B], out_logprobs=self._out_lp[:B])
            return
        logits = self.model.compute_logits(hidden)
        ops.sample(logits, dv["temp"][:B], dv["topk"][:B], dv["topp"][:B], dv["minp"][:B], dv["seeds"][:B],
                   dv["offs"][:B], out_tokens=self._out_tok[:B], out_logprobs=self._out_lp[:B])

    @torch.inference_mode()
    def capture_graphs(self, sizes: list[int] | None = None) -> float:
        if not (self.is_gpu and self.cfg.use_cuda_graph):
            return 0.0
        t0 = time.perf_counter()
        if self._static is None:
            self._alloc_static()
        sizes = sorted(sizes or self.cfg.graph_sizes, reverse=True)
        maxb = self.cfg.max_num_seqs
        sizes = [s for s in sizes if s <= max(maxb, 1)] or [1]
        # dummy inputs: ctx 1, slot -1 (no KV writes), block 0
        self._hv["ctx"].fill_(1)
        self._hv["slots"].fill_(-1)
        self._hv["temp"].fill_(0)
        self._dev_buf.copy_(self._host_buf)
        stream = torch.cuda.Stream(self.device)
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            for _ in range(2):
                self._graph_forward(sizes[0])
        torch.cuda.current_stream().wait_stream(stream)
        torch.cuda.synchronize()
        # No garbage collection while a stream is being captured: a cycle
        # collected mid-capture (e.g. a dead engine's graphs, events and
        # tensors) runs HIP destroy / free calls inside a global-mode capture,
        # which aborts the process.  Collect up front, then hold the GC off.
        gc.collect()
        was_enabled = gc.isenabled()
        gc.disable()
        try:
            for B in sizes:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.graph_pool):
                    self._graph_forward(B)
                if self.graph_pool is None:
                    self.graph_pool = g.pool()
                self.graphs[B] = g
                if self.model.tp.size > 1:  # + the vocab-sharded sampler variant
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=self.graph_pool):
                        self._graph_forward(B, full=False)
                    self.graphs_sharded[B] = g
        finally:
            if was_enabled:
                gc.enable()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def supports_multi_step(self, reqs: list[Request]) -> bool:
        """Whether a pure-decode batch can run as device-chained graph replays."""
        return self._graph_bucket(len(reqs)) is not None and not any(r.params.needs_penalties for r in reqs) and (
            self.model.tp.size == 1 or self._sharded_ok(reqs))

    @torch.inference_mode()
    def execute_decode_multi(self, reqs: list[Request], k: int):
        """k decode steps of `reqs` with one host round trip: the captured
        graph of the batch's bucket is replayed k times and the decode_advance
        kernel feeds each step's sampled tokens, positions, contexts and KV
        slots to the next on the device.  The caller reserved KV slots for k
        tokens per request.  Returns ([k][B] tokens, [k][B] logprobs) or None
        when the batch cannot run this way (no graph bucket, penalties)."""
        B = len(reqs)
        gb = self._graph_bucket(B)
        if gb is None or any(r.params.needs_penalties for r in reqs):
            return None
        t0 = time.perf_counter()
        if self._res_tok is None or self._res_tok.numel() < k * max(self.cfg.graph_sizes):
            n = k * max(self.cfg.graph_sizes)
            self._res_tok = torch.empty(n, dtype=torch.int64, device=self.device)
            self._res_lp = torch.empty(n, dtype=torch.float32, device=self.device)
        self._run_graph(gb, reqs)  # host inputs + H2D + first replay
        dv = self._dv
        kk = ops._k()
        st = ops._stream()
        bt = dv["bt"]
        for i in range(k):
            if i:
                self.graphs[gb].replay()
            kk.decode_advance(dv["ids"].data_ptr(), dv["pos"].data_ptr(), dv["slots"].data_ptr(),
                              dv["ctx"].data_ptr(), dv["offs"].data_ptr(), self._out_tok.data_ptr(),
                              self._out_lp.data_ptr(), self._res_tok.data_ptr(), self._res_lp.data_ptr(),
                              bt.data_ptr(), bt.stride(0), self.block_size, B, i, int(i + 1 < k), st)
        t1 = time.perf_counter()
        toks = self._res_tok[:k * B].view(k, B).tolist()
        lps = self._res_lp[:k * B].view(k, B).tolist()
        tm = self.timing
        tm["decode_prep"] += t1 - t0
        tm["decode_wait"] += time.perf_counter() - t1
        tm["decode_steps"] += k
        tm["decode_seqs"] += k * B
        return toks, lps

    def _next_host_buf(self):
        """The staging buffer for this step's inputs, once its last H2D ran."""
        self._hb ^= 1
        ev = self._h2d_done[self._hb]
        if ev is not None and not ev.query():
            ev.synchronize()
        self._host_buf, self._hv = self._host_bufs[self._hb], self._hvs[self._hb]
        return self._hv

    def _run_graph(self, gb: int, reqs: list[Request], patch=None, prev=None):
        B = len(reqs)
        ids, pos, slots, ctx = self._decode_host_inputs(reqs, gb)
        hv = self._next_host_buf()
        hv["ids"][:gb].numpy()[:] = ids
        hv["pos"][:gb].numpy()[:] = pos
        hv["slots"][:gb].numpy()[:] = slots
        hv["ctx"][:gb].numpy()[:] = ctx
        bt = hv["bt"][:gb].numpy()
        bt[:B] = 0
        for i, r in enumerate(reqs):
            n = len(r.block_ids)
            bt[i, :n] = r.block_ids
        temp, topk, topp, minp, seeds, offs = self._sampling_host(reqs, gb)
        hv["temp"][:gb].numpy()[:] = temp
        hv["topk"][:gb].numpy()[:] = topk
        hv["topp"][:gb].numpy()[:] = topp
        hv["minp"][:gb].numpy()[:] = minp
        hv["seeds"][:gb].numpy()[:] = seeds
        hv["offs"][:gb].numpy()[:] = offs
        self._dev_buf.copy_(self._host_buf, non_blocking=True)
        ev = self._h2d_done[self._hb] = torch.cuda.Event()
        ev.record()
        if patch:  # inputs sampled by the batch still in flight (device to device)
            self._patch_ids(self._dv["ids"], patch, prev)
        g = self.graphs_sharded.get(gb) if self.graphs_sharded and self._sharded_ok(reqs) else None
        (g or self.graphs[gb]).replay()
        return self._out_tok[:B], self._out_lp[:B]
