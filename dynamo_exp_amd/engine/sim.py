"""Timing-faithful engine stand-in (no model, no GPU).

`SimLLMEngine` implements the surface `AsyncLLMEngine` drives (`add_request`,
`abort`, `step`, `has_pending_work`, `requests`, `eos_token_ids`) and spends
each step the way the real engine does on an MI355X: a device phase that
releases the GIL (modelled with `time.sleep`, like a blocking hipStream
synchronize) whose length is `decode_ms` plus the prefill-token cost of the
step's prompt chunks, then the per-step host work of delivering one token per
running stream.  Defaults come from the measured Llama-3-8B bench
(profiles/r1_bench_prefill_dma.json: 15.8 ms decode step at 128 streams with
8192-token chunked prefill).

Use it to measure the serving stack (HTTP frontend, preprocessor, request
plane, router) without a GPU: `run in=http out=sim`, or
`tools/loadgen.py` against it.  The reference has no equivalent in v0.2 (its
echo engines emit tokens on a fixed timer, launch/dynamo-run/src/output/echo_*);
this one keeps the step-synchronous batching of a real engine, which is what
exposes per-step frontend overhead and GIL contention.
"""
from __future__ import annotations

import collections
import os
import time
from types import SimpleNamespace

import torch

from .request import FinishReason, Request, SamplingParams


class SimLLMEngine:
    def __init__(self, decode_ms: float | None = None, prefill_tok_per_ms: float | None = None,
                 max_num_seqs: int = 256, max_batched_tokens: int = 8192, vocab_size: int = 32000,
                 eos_token_ids: list[int] | None = None):
        env = os.environ.get
        self.decode_ms = float(decode_ms if decode_ms is not None else env("DX_SIM_DECODE_MS", "15.0"))
        # mixed steps of the r1 bench: ~105 ms for an 8192-token chunk => ~90 prompt tokens / ms
        self.prefill_tok_per_ms = float(prefill_tok_per_ms if prefill_tok_per_ms is not None
                                        else env("DX_SIM_PREFILL_TOK_PER_MS", "90"))
        # host (GIL-holding) work per step: scheduling, input prep, kernel launches
        self.host_ms = float(env("DX_SIM_HOST_MS", "3.0"))
        self.max_num_seqs = max_num_seqs
        self.max_batched_tokens = max_batched_tokens
        self.vocab_size = vocab_size
        self.eos_token_ids = list(eos_token_ids or [])
        self.model = SimpleNamespace(device=torch.device("cpu"))
        self.requests: dict[str, Request] = {}
        self.waiting: collections.deque[Request] = collections.deque()
        self.running: list[Request] = []
        self.steps = 0
        self.timing = collections.defaultdict(float)

    # -------------------------------------------------------------- requests
    def add_request(self, request_id: str | None, prompt: list[int], params: SamplingParams, on_output=None,
                    remote_prefill: bool = False, remote_decode: bool = False, remote_meta: dict | None = None,
                    mm_embeds=None, mm_hash: int | None = None) -> Request:
        r = Request(request_id or f"sim-{len(self.requests)}", list(prompt), params, on_output=on_output)
        self.requests[r.request_id] = r
        self.waiting.append(r)
        return r

    def abort(self, request_id: str) -> None:
        r = self.requests.get(request_id)
        if r is None:
            return
        r.cancelled = True
        r.finish_reason = FinishReason.CANCELLED
        self._finish(r)

    def has_pending_work(self) -> bool:
        return bool(self.waiting or self.running)

    # ------------------------------------------------------------------ step
    def step(self) -> list[Request]:
        t0 = time.perf_counter()
        budget = self.max_batched_tokens - len(self.running)
        prefill_tokens = 0
        new = []
        while self.waiting and len(self.running) + len(new) < self.max_num_seqs and budget > 0:
            r = self.waiting[0]
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
        device_ms = (self.decode_ms if self.running else 0.0) + prefill_tokens / self.prefill_tok_per_ms
        if device_ms > 0:
            time.sleep(device_ms / 1000.0)  # GIL released, as in a stream synchronize
        self.running.extend(new)
        now = time.perf_counter()
        done = []
        for r in self.running:
            tok = (len(r.prompt) + len(r.output)) % self.vocab_size
            r.output.append(tok)
            r.logprobs.append(0.0)
            if r.first_token_time is None:
                r.first_token_time = now
            p = r.params
            if len(r.output) >= p.max_tokens:
                r.finish_reason = FinishReason.LENGTH
            elif tok in p.stop_token_ids and len(r.output) >= p.min_tokens and not p.ignore_eos:
                r.finish_reason = FinishReason.STOP
            if r.finish_reason is not None:
                done.append(r)
            else:
                self._deliver(r)
        for r in done:
            self._finish(r)
        self.steps += 1
        self.timing["step"] += time.perf_counter() - t0
        return done

    # -------------------------------------------------------------- delivery
    def _finish(self, r: Request) -> None:
        r.finish_time = time.perf_counter()
        if r in self.running:
            self.running.remove(r)
        try:
            self.waiting.remove(r)
        except ValueError:
            pass
        self.requests.pop(r.request_id, None)
        self._deliver(r)

    def _deliver(self, r: Request) -> None:
        new = r.output[r.sent:]
        lps = r.logprobs[r.sent:]
        r.sent = len(r.output)
        fin = r.finish_reason is not None
        if r.on_output is not None and (new or fin):
            r.on_output(r, new, lps, fin)
