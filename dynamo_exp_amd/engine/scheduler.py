"""Continuous-batching scheduler with prefix caching and disaggregation states.

Two policies:

* **chunked** (default, `chunked_prefill=True`): every step is one *mixed*
  batch -- all running streams decode one token, and the rest of the token
  budget (`max_num_batched_tokens`) is filled with prompt chunks (first the
  partially prefilled requests, then newly admitted ones).  On MI355X the
  decode rows ride along in the prefill GEMMs (M grows by ~1%), so the 16 GB
  weight stream of a separate decode step disappears; the budget bounds the
  step time and therefore the inter-token latency.
* **prefill-priority** (`chunked_prefill=False`, what the reference's vLLM
  workers run under disaggregation -- `examples/llm/components/worker.py:72-75`):
  whole prompts are prefilled in their own steps; a decode step is forced every
  `max_prefill_streak` prefill steps.

Requests marked `remote_prefill` only get blocks and park in
REMOTE_PREFILLING (their KV arrives from a prefill worker).  On the prefill
worker, a request whose decode worker already caches a longer prompt prefix
than the local cache (`remote_read_blocks`) parks in READING while those
blocks are pulled, then computes only the rest (the reference's NIXL
read_blocks, Patch:1296-1360).  On KV exhaustion the newest request is
preempted (recompute) back to the waiting queue.
"""
from __future__ import annotations

import time
from collections import deque
from dataclasses import dataclass, field

from .kv_manager import KVManager
from .request import FinishReason, Request, Status


@dataclass
class SchedulerConfig:
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 16384
    max_model_len: int = 8192
    max_prefill_streak: int = 4
    max_prefill_seqs: int = 64
    chunked_prefill: bool = True
    # chunked policy, prefill batching: while streams are decoding and no prompt
    # is part-way through, new prompts wait until `min_prefill_tokens` of them
    # are queued or the oldest has waited `max_prefill_delay` seconds, so the
    # prompt GEMMs run at large M (hipBLASLt: ~1.15-1.35 PFLOP/s at M 3072 vs
    # ~1.5 at M 8192) and the steps in between are graph-replayed decode steps
    min_prefill_tokens: int = 0
    max_prefill_delay: float = 0.0
    # ... and only while at least this many streams decode: a lightly loaded
    # engine has idle time to spare, so holding prompts there only adds TTFT;
    # under load the decode batch grows past it and batching turns itself on
    prefill_hold_min_decode: int = 0
    # ... and the hold also covers the remainder of a prompt split by the
    # token budget: instead of running that remainder (plus whatever queued
    # meanwhile) as a small step right away, it waits with the queue until
    # min_prefill_tokens are available or its request has waited
    # max_prefill_delay since it arrived -- fewer, fuller mixed steps; only
    # while at least this many streams decode (0 = off): a saturated engine
    # trades TTFT for full-tile GEMMs, a moderately loaded one keeps its TTFT
    prefill_hold_partial: int = 0
    # chunked policy: once a step's prompt chunks fill half the budget, a new
    # prompt that does not fit whole waits for the next step (which it leads,
    # past any hold) instead of being split -- a split leaves a remainder of a
    # few hundred tokens that often runs as a small, tile-starved mixed step
    # of its own -- measured -3.5 % (profiles/r4_prefill_hold_partial_ab.txt)
    prefill_whole_prompts: bool = False


PLACEHOLDER = -1  # output slot of a token sampled on the device, not yet read back


@dataclass
class Batch:
    """requests[:n_prefill] compute prompt chunks (num_new[i] tokens each;
    `sample[i]` when the chunk completes the prompt), the rest decode one token.
    kind: "prefill" (no decode rows) | "decode" (no prefill rows) | "mixed"."""

    kind: str
    requests: list[Request]
    num_new: list[int] = field(default_factory=list)
    sample: list[bool] = field(default_factory=list)
    epochs: list[int] = field(default_factory=list)  # async: Request.epoch of `sampled` at launch

    @property
    def n_prefill(self) -> int:
        return len(self.num_new)

    @property
    def num_tokens(self) -> int:
        return sum(self.num_new) + len(self.requests) - len(self.num_new)

    @property
    def sampled(self) -> list[Request]:
        """Requests that produce a token this step, in logits-row order."""
        n = self.n_prefill
        return [r for r, s in zip(self.requests[:n], self.sample) if s] + self.requests[n:]


class Scheduler:
    def __init__(self, cfg: SchedulerConfig, kv: KVManager):
        self.cfg = cfg
        self.kv = kv
        self.waiting: deque[Request] = deque()
        self.running: list[Request] = []
        self.prefilling: list[Request] = []  # admitted, prompt partially computed (chunked)
        self.remote: dict[str, Request] = {}  # REMOTE_PREFILLING on the decode side
        self.transferring: dict[str, Request] = {}  # prefill side: KV handed to a decode worker
        self.reading: dict[str, Request] = {}  # prefill side: pulling a cached prefix (READ path)
        # decode side, one-sided (IPC) KV transport: remote prefills whose KV a
        # prefill worker may be writing straight into their blocks, and the ones
        # aborted meanwhile, whose blocks are held until that write is done
        self.write_pending: set[str] = set()
        self.write_zombies: dict[str, Request] = {}
        # decode side, one-sided transport: requests whose cached prefix blocks a
        # prefill worker is reading (READ) -- held like write_pending
        self.read_pinned: set[str] = set()
        self._streak = 0
        self.preemptions = 0
        self._deferred_whole = False  # a prompt was left for the next step (prefill_whole_prompts)
        # time source of the prefill-batching hold decision.  Under tensor
        # parallelism every rank runs its own copy of this scheduler, so the
        # ReplicatedEngine replaces it with the leader's broadcast step time:
        # a per-process wall clock would let ranks disagree about releasing
        # held prompts and enter the collectives with different batches.
        self.clock = time.perf_counter
        self.on_remote_prefill = None  # callback(req) when a remote-prefill request got its blocks
        # callback(req, first_block, last_block): pull blocks [first, last) of the
        # prompt from the decode worker, then call finish_remote_read
        self.on_remote_read = None

    # ------------------------------------------------------------------ queue
    def add(self, req: Request) -> None:
        if len(req.prompt) + 1 > self.cfg.max_model_len:
            raise ValueError(f"prompt of {len(req.prompt)} tokens exceeds max_model_len {self.cfg.max_model_len}")
        req.status = Status.WAITING
        req.sched_arrival = self.clock()
        self.waiting.append(req)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or self.prefilling)

    def num_unfinished(self) -> int:
        return len(self.waiting) + len(self.running) + len(self.prefilling) + len(self.remote) + \
            len(self.transferring) + len(self.reading)

    def num_active(self) -> int:
        return len(self.running) + len(self.prefilling) + len(self.remote) + len(self.reading)

    def abort(self, request_id: str) -> Request | None:
        for q in (self.running, self.prefilling, self.waiting):
            for r in list(q):
                if r.request_id == request_id:
                    q.remove(r)
                    self._finish(r, FinishReason.CANCELLED)
                    return r
        for table in (self.remote, self.reading):
            r = table.pop(request_id, None)
            if r is not None:
                # (a remote prefill a peer may be writing into keeps its blocks: _finish)
                self._finish(r, FinishReason.CANCELLED)
                return r
        return None

    def release_write(self, request_id: str) -> bool:
        """One-sided transport: the write into an aborted request's blocks is
        over (its "done" or "fail" arrived): free them now."""
        self.write_pending.discard(request_id)
        return self._free_zombie(request_id)

    def unpin_read(self, request_id: str) -> bool:
        """One-sided transport: a prefill worker finished reading this
        request's prefix blocks; free them if the request finished meanwhile."""
        self.read_pinned.discard(request_id)
        return self._free_zombie(request_id)

    def _free_zombie(self, request_id: str) -> bool:
        if request_id in self.write_pending or request_id in self.read_pinned:
            return False
        r = self.write_zombies.pop(request_id, None)
        if r is None:
            return False
        self.kv.free(r)
        return True

    def _park_for_read(self, r: Request) -> bool:
        """After allocate_prompt: if the decode worker holds more of the
        prompt's prefix than the local cache, pull it (READING) instead of
        recomputing it.  The waiting-queue head `r` is consumed when True."""
        if not r.remote_read_blocks or self.on_remote_read is None:
            return False
        bs = self.kv.block_size
        have = r.num_computed // bs
        want = min(r.remote_read_blocks, (len(r.prompt) - 1) // bs)  # >= 1 token left to compute
        if want <= have:
            return False
        self.waiting.popleft()
        r.admit_time = time.perf_counter()
        r.status = Status.READING
        r.read_upto = want
        self.reading[r.request_id] = r
        self.on_remote_read(r, have, want)
        return True

    def finish_remote_read(self, request_id: str, ok: bool = True) -> Request | None:
        """Prefill side: the pulled prefix landed in the request's blocks;
        register it in the local prefix cache and compute the rest.  ok=False:
        the decode worker no longer held those blocks (it had given the
        request up and sent filler bytes), so nothing is registered and the
        prefix is recomputed from the local cache hit on."""
        r = self.reading.pop(request_id, None)
        if r is None:
            return None
        if ok:
            r.num_computed = r.read_upto * self.kv.block_size
            self.kv.register_filled(r)
        else:
            r.remote_read_blocks = 0
        r.status = Status.RUNNING
        if self.cfg.chunked_prefill:
            self.prefilling.append(r)
        else:
            r.kv_ready = True
            self.waiting.appendleft(r)
        return r

    # ------------------------------------------------------------------ schedule
    def schedule(self) -> Batch | None:
        cfg = self.cfg
        if cfg.chunked_prefill:
            return self._schedule_chunked()
        prefill_ok = self.waiting and (self._streak < cfg.max_prefill_streak or not self.running)
        if prefill_ok:
            batch = self._schedule_prefill()
            if batch is not None:
                self._streak += 1
                return batch
        self._streak = 0
        if not self.running:
            return None
        return self._schedule_decode()

    def _schedule_prefill(self) -> Batch | None:
        cfg = self.cfg
        reqs, news = [], []
        budget = cfg.max_num_batched_tokens
        while self.waiting and len(self.running) + len(reqs) < cfg.max_num_seqs and len(reqs) < cfg.max_prefill_seqs:
            r = self.waiting[0]
            if r.cancelled:
                self.waiting.popleft()
                self._finish(r, FinishReason.CANCELLED)
                continue
            if r.remote_prefill:
                if not self.kv.allocate_for_remote(r):
                    break
                self.waiting.popleft()
                r.admit_time = time.perf_counter()
                r.status = Status.REMOTE_PREFILLING
                self.remote[r.request_id] = r
                if self.on_remote_prefill is not None:
                    self.on_remote_prefill(r)
                continue
            if r.kv_ready:  # blocks allocated and prefix pulled (READ path)
                if reqs and len(r.prompt) - r.num_computed > budget:
                    break
            else:
                # token budget is checked before allocation (estimate with cached prefix)
                hp = r.hash_prompt if r.hash_prompt is not None else r.prompt
                est_new = len(r.prompt) - self.kv.prefix_hit_tokens_for(hp) if self.kv.caching else len(r.prompt)
                est_new = max(1, est_new)
                if reqs and est_new > budget:
                    break
                if not self.kv.allocate_prompt(r):
                    break
                if self._park_for_read(r):
                    continue
            self.waiting.popleft()
            r.admit_time = time.perf_counter()
            n_new = len(r.prompt) - r.num_computed
            budget -= n_new
            r.status = Status.RUNNING
            reqs.append(r)
            news.append(n_new)
            if budget <= 0:
                break
        if not reqs:
            return None
        return Batch("prefill", reqs, news, [True] * len(reqs))

    def _admit(self, r: Request) -> bool:
        """Waiting-queue head handling shared by both policies; True if `r`
        was consumed (cancelled / parked for remote prefill)."""
        if r.cancelled:
            self.waiting.popleft()
            self._finish(r, FinishReason.CANCELLED)
            return True
        return False

    def _schedule_chunked(self) -> Batch | None:
        cfg = self.cfg
        decode = self._collect_decode()
        budget = cfg.max_num_batched_tokens - len(decode)
        pre, news, samp = [], [], []
        deferred, self._deferred_whole = self._deferred_whole, False
        # (a prompt deferred by prefill_whole_prompts leads this step past any hold: ADVICE r4)
        if (cfg.prefill_hold_partial and cfg.min_prefill_tokens > 0 and decode and self.prefilling and not deferred
                and len(decode) >= max(cfg.prefill_hold_min_decode, cfg.prefill_hold_partial)
                and self._hold_prefill(partial=True)):
            return Batch("decode", decode)
        for r in list(self.prefilling):
            if budget <= 0 or len(pre) >= cfg.max_prefill_seqs:
                break
            if r.cancelled:
                self.prefilling.remove(r)
                self._finish(r, FinishReason.CANCELLED)
                continue
            n = min(len(r.prompt) - r.num_computed, budget)
            pre.append(r)
            news.append(n)
            samp.append(r.num_computed + n == len(r.prompt))
            budget -= n
        hold = (cfg.min_prefill_tokens > 0 and decode and len(decode) >= cfg.prefill_hold_min_decode and not pre
                and not deferred and self._hold_prefill())
        while not hold and self.waiting and budget > 0 and len(pre) < cfg.max_prefill_seqs and \
                len(self.running) + len(self.prefilling) < cfg.max_num_seqs:
            r = self.waiting[0]
            if self._admit(r):
                continue
            if (cfg.prefill_whole_prompts and not r.remote_prefill and len(r.prompt) - r.num_computed > budget
                    and cfg.max_num_batched_tokens - len(decode) - budget >= cfg.max_num_batched_tokens // 2):
                self._deferred_whole = True
                break
            if r.remote_prefill:
                if not self.kv.allocate_for_remote(r):
                    break
                self.waiting.popleft()
                r.admit_time = time.perf_counter()
                r.status = Status.REMOTE_PREFILLING
                self.remote[r.request_id] = r
                if self.on_remote_prefill is not None:
                    self.on_remote_prefill(r)
                continue
            if not self.kv.allocate_prompt(r):
                break
            if self._park_for_read(r):
                continue
            self.waiting.popleft()
            r.admit_time = time.perf_counter()
            r.status = Status.RUNNING
            self.prefilling.append(r)
            n = min(len(r.prompt) - r.num_computed, budget)
            pre.append(r)
            news.append(n)
            samp.append(r.num_computed + n == len(r.prompt))
            budget -= n
        if not pre and not decode:
            return None
        kind = "mixed" if pre and decode else ("prefill" if pre else "decode")
        return Batch(kind, pre + decode, news, samp)

    def _hold_prefill(self, partial: bool = False) -> bool:
        """Prefill batching (min_prefill_tokens / max_prefill_delay): True
        while queued local prompts are too few and none has waited too long.
        Remote-prefill requests at the head are never held.  partial: the
        part-computed prompts count as queued (and as the oldest)."""
        cfg = self.cfg
        head = self.waiting[0] if self.waiting else None
        if head is not None and (head.remote_prefill or head.cancelled):
            return False
        if partial and self.prefilling:  # the oldest of the split prompt and the queue head (a re-queued
            # preempted request can be older than the prompt in flight)
            p = self.prefilling[0]
            if p.cancelled:
                return False
            head = p if head is None or p.sched_arrival <= head.sched_arrival else head
        if head is None:
            return False
        if self.clock() - head.sched_arrival >= cfg.max_prefill_delay:
            return False
        queued = 0
        for r in (self.prefilling + list(self.waiting) if partial else self.waiting):
            queued += len(r.prompt) - r.num_computed
            if queued >= cfg.min_prefill_tokens:
                return False
        return True

    def _schedule_decode(self) -> Batch | None:
        batch = self._collect_decode()
        if not batch:
            return None
        return Batch("decode", batch)

    def _collect_decode(self) -> list[Request]:
        """All running streams that could grow by one token (preempting the
        newest ones when the KV pool is exhausted)."""
        cfg = self.cfg
        batch: list[Request] = []
        preempted: set[str] = set()
        for r in list(self.running):
            if r.request_id in preempted:
                continue  # a victim of an earlier stream's growth this step
            if r.cancelled:
                self.running.remove(r)
                self._finish(r, FinishReason.CANCELLED)
                continue
            if r.pending and (len(r.output) >= r.params.max_tokens or r.num_tokens >= cfg.max_model_len):
                continue  # async: every token it may produce is already in flight
            # slot for the token produced by this step's input (already counted
            # in num_tokens): need capacity for num_tokens tokens
            while not self.kv.ensure_slots(r, r.num_tokens):
                victim = self.running[-1]
                if victim is r:
                    break
                self._preempt(victim)
                preempted.add(victim.request_id)
            else:
                batch.append(r)
                continue
            # could not grow even after preempting everyone after it
            self._preempt(r)
        return batch[: cfg.max_num_seqs]

    def _preempt(self, r: Request) -> None:
        if r in self.running:
            self.running.remove(r)
        if r in self.prefilling:
            self.prefilling.remove(r)
        self.kv.free(r)
        if r.pending:  # async: tokens still on the device are dropped (recomputed later)
            del r.output[len(r.output) - r.pending:]
            del r.logprobs[len(r.logprobs) - r.pending:]
            r.sample_offset -= r.pending
            r.pending = 0
        r.epoch += 1
        # recompute: fold generated tokens into the prompt
        if r.hash_prompt is not None:
            r.hash_prompt = r.hash_prompt + r.output
        r.prompt = r.prompt + r.output
        r.params.max_tokens = max(1, r.params.max_tokens - len(r.output))
        r.params.min_tokens = max(0, r.params.min_tokens - len(r.output))
        r.sent -= len(r.output)
        r.output = []
        r.logprobs = []
        r.num_computed = 0
        r.kv_ready = False
        r.block_hashes, r.seq_hashes = [], []
        r.status = Status.WAITING
        self.waiting.appendleft(r)
        self.preemptions += 1
        r.preempted = getattr(r, "preempted", 0) + 1

    def fallback_local(self, request_id: str) -> Request | None:
        """Decode side: give up on a remote prefill whose KV transfer never
        started (the prefill worker failed or died first) and compute the
        prompt here.  Its blocks are already allocated, its cached prefix
        counted; it continues like a pulled-prefix request."""
        r = self.remote.pop(request_id, None)
        if r is None:
            return None
        self.write_pending.discard(request_id)
        r.remote_prefill = False
        r.status = Status.RUNNING
        if self.cfg.chunked_prefill:
            self.prefilling.append(r)
        else:
            r.kv_ready = True
            self.waiting.appendleft(r)
        self.fallbacks = getattr(self, "fallbacks", 0) + 1
        return r

    # ------------------------------------------------------------------ results
    def finish_remote_prefill(self, request_id: str, first_token: int | None, first_logprob: float = 0.0) -> Request | None:
        """Decode side: the remote KV landed; join the running batch."""
        self.write_pending.discard(request_id)
        r = self.remote.pop(request_id, None)
        if r is None:
            return None
        r.num_computed = len(r.prompt)
        self.kv.register_filled(r)
        r.status = Status.RUNNING
        if first_token is not None:
            self._append_token(r, first_token, first_logprob)
            if r.finished:
                return r
        self.running.append(r)
        return r

    def update(self, batch: Batch, tokens: list[int], logprobs: list[float] | None = None) -> list[Request]:
        """Apply one step; `tokens` are in `batch.sampled` order.  Returns the
        requests that produced output."""
        out = []
        ti = 0
        n_pre = batch.n_prefill
        for i, r in enumerate(batch.requests):
            if i < n_pre:
                r.num_computed += batch.num_new[i]
                self.kv.register_filled(r)
                if not batch.sample[i]:
                    continue  # partial prompt chunk: no token yet
                if r in self.prefilling:
                    self.prefilling.remove(r)
                tok, lp = tokens[ti], (logprobs[ti] if logprobs else 0.0)
                ti += 1
                if r.remote_decode:
                    # prefill worker: first token goes to the decode worker along with the KV
                    self._append_token(r, tok, lp, count_only=True)
                    r.status = Status.TRANSFERRING
                    self.transferring[r.request_id] = r
                    out.append(r)
                    continue
                self.running.append(r)
            else:
                r.num_computed = r.num_tokens
                self.kv.register_filled(r)
                tok, lp = tokens[ti], (logprobs[ti] if logprobs else 0.0)
                ti += 1
            self._append_token(r, tok, lp)
            out.append(r)
        return out

    # ------------------------------------------------------------------ asynchronous scheduling
    def pre_update(self, batch: Batch) -> None:
        """A batch was launched and its tokens are not read back yet: apply
        everything that does not depend on their values, so the next batch can
        be scheduled while this one runs on the GPU -- KV progress, prompts that
        complete join the running set, and each sampled row gets a placeholder
        output token (its value arrives with `update_async`)."""
        n_pre = batch.n_prefill
        batch.epochs = [r.epoch for r in batch.sampled]
        for i, r in enumerate(batch.requests):
            if i < n_pre:
                r.num_computed += batch.num_new[i]
                if not batch.sample[i]:
                    continue
                if r in self.prefilling:
                    self.prefilling.remove(r)
                if r.remote_decode:
                    continue  # the first token leaves with the KV (update_async)
                self.running.append(r)
            else:
                r.num_computed = r.num_tokens
            r.output.append(PLACEHOLDER)
            r.logprobs.append(0.0)
            r.sample_offset += 1
            r.pending += 1

    def update_async(self, batch: Batch, tokens: list[int], logprobs: list[float] | None = None) -> list[Request]:
        """The tokens of a batch launched earlier (after pre_update): fill in
        the placeholders, register filled blocks, apply stop conditions.  A
        request that finished (or was preempted) since drops its stale token;
        one that finishes now drops the placeholders of later batches."""
        out = []
        for k, r in enumerate(batch.sampled):
            tok, lp = int(tokens[k]), (float(logprobs[k]) if logprobs else 0.0)
            if r.finished or r.epoch != batch.epochs[k]:
                continue
            if r.remote_decode and r.status == Status.RUNNING and not r.pending:
                # prefill worker: first token goes to the decode worker along with the KV
                self.kv.register_filled(r)
                self._append_token(r, tok, lp, count_only=True)
                r.status = Status.TRANSFERRING
                self.transferring[r.request_id] = r
                out.append(r)
                continue
            idx = len(r.output) - r.pending
            r.output[idx] = tok
            r.logprobs[idx] = lp
            r.pending -= 1
            self.kv.register_filled(r)
            p = r.params
            n = idx + 1
            reason = None
            if n >= p.max_tokens:
                reason = FinishReason.LENGTH
            elif n >= p.min_tokens and tok in p.stop_token_ids:
                reason = FinishReason.STOP
            elif len(r.prompt) + n >= self.cfg.max_model_len:
                reason = FinishReason.LENGTH
            if reason is not None:
                if r.pending:  # tokens sampled after the stop are discarded
                    del r.output[n:]
                    del r.logprobs[n:]
                    r.pending = 0
                if r in self.running:
                    self.running.remove(r)
                self._finish(r, reason)
            out.append(r)
        return out

    # ------------------------------------------------------------------ multi-step decode
    def reserve_multi(self, batch: Batch, k: int) -> int:
        """Steps a pure-decode batch may run back to back without the host
        (engine multi-step): only while nothing waits for admission (new
        prompts would otherwise wait k steps), bounded by max_model_len, with
        KV slots reserved for every step up front.  Returns 1 when not
        applicable."""
        if k <= 1 or batch.kind != "decode" or self.waiting or self.prefilling:
            return 1
        k = min(k, min(self.cfg.max_model_len - r.num_tokens + 1 for r in batch.requests))
        if k <= 1:
            return 1
        for r in batch.requests:
            if not self.kv.ensure_slots(r, r.num_tokens + k - 1):
                return 1  # slots reserved so far stay with their requests (used by later steps)
        return k

    def update_multi(self, batch: Batch, tokens: list[list[int]], logprobs: list[list[float]]) -> list[Request]:
        """Apply k decode steps (tokens[i][j]: step i, request j).  A request
        that finishes at step i ignores its later tokens (computed on the
        device before the host saw the stop)."""
        out, seen = [], set()
        for toks, lps in zip(tokens, logprobs):
            for j, r in enumerate(batch.requests):
                if r.finished or r.status != Status.RUNNING:
                    continue
                r.num_computed = r.num_tokens
                self.kv.register_filled(r)
                self._append_token(r, toks[j], lps[j])
                if r.request_id not in seen:
                    seen.add(r.request_id)
                    out.append(r)
        return out

    def finish_transfer(self, request_id: str) -> Request | None:
        r = self.transferring.pop(request_id, None)
        if r is not None:
            self._finish(r, FinishReason.REMOTE_DECODE)
        return r

    def _append_token(self, r: Request, tok: int, lp: float, count_only: bool = False) -> None:
        r.output.append(int(tok))
        r.logprobs.append(float(lp))
        r.sample_offset += 1
        if count_only:
            return
        p = r.params
        n = len(r.output)
        reason = None
        if n >= p.max_tokens:
            reason = FinishReason.LENGTH
        elif n >= p.min_tokens and int(tok) in p.stop_token_ids:
            reason = FinishReason.STOP
        elif r.num_tokens >= self.cfg.max_model_len:
            reason = FinishReason.LENGTH
        if reason is not None:
            if r in self.running:
                self.running.remove(r)
            self._finish(r, reason)

    def _finish(self, r: Request, reason: FinishReason) -> None:
        r.status = Status.FINISHED
        r.finish_reason = reason
        r.finish_time = time.perf_counter()
        if r.request_id in self.write_pending or r.request_id in self.read_pinned:
            # one-sided KV transport: a prefill worker may still be writing into
            # these blocks (aborted remote prefill, or one that timed out and was
            # prefilled here): hold them until release_write()
            self.write_zombies[r.request_id] = r
            return
        self.kv.free(r)
