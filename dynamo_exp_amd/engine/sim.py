"""Timing-faithful engine stand-in (no model, no GPU).

`SimLLMEngine` implements the surface the serving stack drives
(`add_request`, `abort`, `step`, `has_pending_work`, `requests`,
`eos_token_ids`, `forward_pass_metrics`, the disaggregation hooks) and
spends each step the way the real engine does on an MI355X: a device phase
that releases the GIL (modelled with `time.sleep`, like a blocking hipStream
synchronize) whose length is the decode cost of the running batch plus the
prefill-token cost of the step's prompt chunks, then the per-step host work
of delivering one token per running stream.

Roles (disaggregation):
* decode engine: a `remote_prefill` request gets its blocks, parks, and the
  scheduler callback `on_remote_prefill(req)` fires (the worker enqueues a
  RemotePrefillRequest); `finish_remote_prefill(rid, tok, lp)` (when the KV
  "landed", disagg/sim_agent.py) moves it into the decode batch;
* prefill engine: a `remote_decode` request is prefilled, its first token
  sampled, `prefill_done_hook(req)` fires and its blocks are released.

Calibration (`SimLLMEngine.mi355x_8b`): the measured Llama-3-8B TP1 roles on
one MI355X (profiles/r2_role_capacities.txt): prefill 94.7k prompt tok/s;
decode 22.9 ms per step at 256 streams of ~3k context, ~6.5 ms weight-stream
floor at small batch (profiles/r2_step_breakdown_session3.txt) -> 6.5 ms +
0.064 ms per running stream; KV blocks for 0.9 of 288 GB.  Generic defaults
(`decode_ms` fixed per step) keep the old behaviour for frontend studies
(`run in=http out=sim`, tools/loadgen.py).

The reference has no equivalent in v0.2 (its echo engines emit tokens on a
fixed timer, lib/llm/src/engines.rs:67-160); this one keeps the
step-synchronous batching and the load signals (slots, KV usage, queue) the
router and the planner react to.
"""
from __future__ import annotations

import collections
import os
import time
from types import SimpleNamespace

import torch

from .request import FinishReason, Request, SamplingParams, Status


class SimLLMEngine:
    def __init__(self, decode_ms: float | None = None, prefill_tok_per_ms: float | None = None,
                 max_num_seqs: int = 256, max_batched_tokens: int = 8192, vocab_size: int = 32000,
                 eos_token_ids: list[int] | None = None, decode_per_seq_ms: float | None = None,
                 num_blocks: int | None = None, block_size: int = 64, host_ms: float | None = None):
        env = os.environ.get
        self.decode_ms = float(decode_ms if decode_ms is not None else env("DX_SIM_DECODE_MS", "15.0"))
        self.decode_per_seq_ms = float(decode_per_seq_ms if decode_per_seq_ms is not None
                                       else env("DX_SIM_DECODE_PER_SEQ_MS", "0"))
        # mixed steps of the r1 bench: ~105 ms for an 8192-token chunk => ~90 prompt tokens / ms
        self.prefill_tok_per_ms = float(prefill_tok_per_ms if prefill_tok_per_ms is not None
                                        else env("DX_SIM_PREFILL_TOK_PER_MS", "90"))
        # host (GIL-holding) work per step: scheduling, input prep, kernel launches
        self.host_ms = float(host_ms if host_ms is not None else env("DX_SIM_HOST_MS", "3.0"))
        self.max_num_seqs = max_num_seqs
        self.max_batched_tokens = max_batched_tokens
        self.vocab_size = vocab_size
        self.eos_token_ids = list(eos_token_ids or [])
        self.model = SimpleNamespace(device=torch.device("cpu"), cfg=SimpleNamespace(num_key_value_heads=8))
        self.model_cfg = SimpleNamespace(vocab_size=vocab_size, name="sim")
        self.cfg = SimpleNamespace(max_num_seqs=max_num_seqs, max_num_batched_tokens=max_batched_tokens)
        self.block_size = block_size
        self.num_blocks = int(num_blocks or 1 << 20)
        self.kv = SimpleNamespace(block_size=block_size, hit_rate=lambda: 0.0, num_blocks=self.num_blocks)
        self.requests: dict[str, Request] = {}
        self.waiting: collections.deque[Request] = collections.deque()
        self.running: list[Request] = []
        self.remote: dict[str, Request] = {}  # decode side: parked while the prefill happens elsewhere
        self.scheduler = SimpleNamespace(on_remote_prefill=None, on_remote_read=None, remote=self.remote,
                                         reading={}, transferring={}, waiting=self.waiting)
        self.prefill_done_hook = None
        self.batch_hook = None
        self.steps = 0
        self.stats = dict(steps=0, prefill_steps=0, decode_steps=0, mixed_steps=0, prompt_tokens=0,
                          generated_tokens=0)
        self.timing = collections.defaultdict(float)
        from ..utils.tracing import RequestTimer

        self.request_timer = RequestTimer()

    @classmethod
    def mi355x_8b(cls, role: str = "decode", slowdown: float = 1.0, gpu_gb: float = 288.0, **kw) -> "SimLLMEngine":
        """Llama-3-8B TP1 on one MI355X (see the module docstring).
        `slowdown` k > 1 models a GPU k times slower (device step times x k,
        prefill rate / k) and `gpu_gb` its memory (KV pool): the planner
        benchmark's overload regime (the reference's 8x
        H100 runs overloaded static 2P2D at the trace's peak)."""
        per_block = 32 * 2 * 8 * 64 * 128 * 2  # bytes of one 64-token block, all layers, K and V
        util = 0.5 if role == "prefill" else 0.9
        blocks = int((gpu_gb * 1e9 * util - 16e9 - 6e9) // per_block)
        if blocks <= 0:
            raise ValueError(f"sim: {gpu_gb} GB leaves no KV blocks")
        k = float(slowdown)
        d = dict(decode_ms=6.5 * k, decode_per_seq_ms=0.064 * k, prefill_tok_per_ms=94.7 / k, host_ms=1.0,
                 max_num_seqs=32 if role == "prefill" else 256,
                 max_batched_tokens=16384 if role == "prefill" else 8192, num_blocks=blocks, block_size=64,
                 vocab_size=128256, eos_token_ids=[128001])
        d.update(kw)
        return cls(**d)

    # -------------------------------------------------------------- requests
    def add_kv_event_listener(self, fn) -> None:  # no prefix cache: no KV events
        pass

    def add_request(self, request_id: str | None, prompt: list[int], params: SamplingParams, on_output=None,
                    remote_prefill: bool = False, remote_decode: bool = False, remote_meta: dict | None = None,
                    mm_embeds=None, mm_hash: int | None = None, remote_read_blocks: int = 0) -> Request:
        r = Request(request_id or f"sim-{len(self.requests)}", list(prompt), params, on_output=on_output,
                    remote_prefill=remote_prefill, remote_decode=remote_decode, remote_meta=remote_meta or {})
        self.requests[r.request_id] = r
        self.waiting.append(r)
        self.stats["prompt_tokens"] += len(prompt)
        return r

    def abort(self, request_id: str) -> None:
        r = self.requests.get(request_id)
        if r is None:
            return
        r.cancelled = True
        r.finish_reason = FinishReason.CANCELLED
        self.remote.pop(request_id, None)
        self._finish(r)

    def has_pending_work(self) -> bool:
        return bool(self.waiting or self.running)

    def has_unfinished(self) -> bool:
        return bool(self.waiting or self.running or self.remote)

    def _blocks(self, r: Request) -> int:
        return -(-(len(r.prompt) + len(r.output)) // self.block_size)

    def forward_pass_metrics(self) -> dict:
        """The reference ForwardPassMetrics fields (router / planner signals)."""
        used = sum(self._blocks(r) for r in self.running) + sum(self._blocks(r) for r in self.remote.values())
        used += sum(-(-r.num_computed // self.block_size) for r in self.waiting)
        return dict(request_active_slots=len(self.running) + len(self.remote),
                    request_total_slots=self.max_num_seqs, kv_active_blocks=used, kv_total_blocks=self.num_blocks,
                    num_requests_waiting=len(self.waiting), gpu_cache_usage_perc=used / max(1, self.num_blocks),
                    gpu_prefix_cache_hit_rate=0.0)

    # ------------------------------------------------------------------ step
    def step(self) -> list[Request]:
        t0 = time.perf_counter()
        budget = self.max_batched_tokens - len(self.running)
        prefill_tokens = 0
        new = []
        slots = len(self.running) + len(self.remote)
        while self.waiting and slots + len(new) < self.max_num_seqs and budget > 0:
            r = self.waiting[0]
            if r.remote_prefill:  # decode side: blocks now, the prefill happens elsewhere
                self.waiting.popleft()
                r.admit_time = time.perf_counter()
                r.status = Status.REMOTE_PREFILLING
                self.remote[r.request_id] = r
                slots += 1
                if self.scheduler.on_remote_prefill is not None:
                    self.scheduler.on_remote_prefill(r)
                continue
            if r.admit_time is None:
                r.admit_time = time.perf_counter()
            left = len(r.prompt) - r.num_computed
            take = min(left, budget)
            r.num_computed += take
            prefill_tokens += take
            budget -= take
            if r.num_computed < len(r.prompt):
                break  # chunked: the rest of the prompt goes in the next step
            self.waiting.popleft()
            new.append(r)
        t_host = time.perf_counter() + self.host_ms / 1000.0
        while time.perf_counter() < t_host:  # pure-Python busy work holds the GIL
            pass
        B = len(self.running)
        device_ms = (self.decode_ms + self.decode_per_seq_ms * B if B else 0.0) + \
            prefill_tokens / self.prefill_tok_per_ms
        if device_ms > 0:
            time.sleep(device_ms / 1000.0)  # GIL released, as in a stream synchronize
        self.timing["device"] += device_ms / 1000.0
        kind = "mixed" if (B and prefill_tokens) else ("prefill" if prefill_tokens else "decode")
        if B or prefill_tokens:
            self.stats["steps"] += 1
            self.stats[f"{kind}_steps"] += 1
        now = time.perf_counter()
        done = []
        for r in new:
            if r.remote_decode:  # prefill side: first token, hand the KV off, release the blocks
                r.output.append((len(r.prompt) * 31) % self.vocab_size)
                r.logprobs.append(0.0)
                r.first_token_time = now
                r.finish_reason = FinishReason.REMOTE_DECODE
                if self.prefill_done_hook is not None:
                    self.prefill_done_hook(r)
                self._finish(r)
                continue
            self.running.append(r)
        for r in self.running:
            self._emit_token(r, now)
            if r.finish_reason is not None:
                done.append(r)
            else:
                self._deliver(r)
        for r in done:
            self._finish(r)
        self.steps += 1
        self.timing["step"] += time.perf_counter() - t0
        return done

    def _emit_token(self, r: Request, now: float) -> None:
        tok = (len(r.prompt) + len(r.output)) % self.vocab_size
        r.output.append(tok)
        r.logprobs.append(0.0)
        self.stats["generated_tokens"] += 1
        if r.first_token_time is None:
            r.first_token_time = now
        p = r.params
        if len(r.output) >= p.max_tokens:
            r.finish_reason = FinishReason.LENGTH
        elif tok in p.stop_token_ids and len(r.output) >= p.min_tokens and not p.ignore_eos:
            r.finish_reason = FinishReason.STOP

    # -------------------------------------------------------------- disaggregation
    def finish_remote_prefill(self, request_id: str, first_token: int | None, logprob: float = 0.0) -> None:
        """Decode side: the remote KV landed; the request joins the batch with
        the prefill worker's first token."""
        r = self.remote.pop(request_id, None)
        if r is None:
            return
        r.num_computed = len(r.prompt)
        if first_token is not None:
            r.output.append(int(first_token))
            r.logprobs.append(float(logprob))
            self.stats["generated_tokens"] += 1
        r.first_token_time = time.perf_counter()
        if len(r.output) >= r.params.max_tokens:
            r.finish_reason = FinishReason.LENGTH
            self._finish(r)
            return
        self.running.append(r)
        self._deliver(r)

    def finish_transfer(self, request_id: str) -> None:  # blocks were released at the handoff
        pass

    def finish_remote_read(self, request_id: str) -> None:  # no prefix cache, nothing is ever read
        pass

    # -------------------------------------------------------------- delivery
    def _finish(self, r: Request) -> None:
        r.finish_time = time.perf_counter()
        r.status = Status.FINISHED
        if r in self.running:
            self.running.remove(r)
        try:
            self.waiting.remove(r)
        except ValueError:
            pass
        self.requests.pop(r.request_id, None)
        self._deliver(r)
        if r.finish_reason not in (FinishReason.REMOTE_DECODE, FinishReason.CANCELLED):
            self.request_timer.observe(r)

    def _deliver(self, r: Request) -> None:
        new = r.output[r.sent:]
        lps = r.logprobs[r.sent:]
        r.sent = len(r.output)
        fin = r.finish_reason is not None
        if r.on_output is not None and (new or fin):
            r.on_output(r, new, lps, fin)
