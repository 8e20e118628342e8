"""Backend operator: incremental detokenization + stop handling between the
token-level engine and the preprocessor (reference lib/llm/src/backend.rs).

* hidden stop token ids are enforced by the engine; here we enforce stop
  *strings* with a "jail": text that could still become a stop string is held
  back until it can be released or matched (backend.rs:274-430);
* on a stop-string match the output is truncated, finish_reason = "stop" and
  the upstream engine is asked to stop (`Context.stop_generating`);
* detokenization is O(1) per token (DecodeStream window).
"""
from __future__ import annotations

from typing import AsyncIterator, Callable

from ..runtime.context import Context
from .tokenizer import Tokenizer


class StopJail:
    def __init__(self, stops: list[str]):
        self.stops = [s for s in stops if s]
        self.buf = ""
        self.max_len = max((len(s) for s in self.stops), default=0)

    def push(self, text: str) -> tuple[str, bool]:
        """Returns (releasable text, matched)."""
        if not self.stops:
            return text, False
        self.buf += text
        best = None
        for s in self.stops:
            i = self.buf.find(s)
            if i >= 0 and (best is None or i < best):
                best = i
        if best is not None:
            out = self.buf[:best]
            self.buf = ""
            return out, True
        # hold back the longest suffix that is a prefix of some stop string
        hold = 0
        for k in range(1, min(self.max_len, len(self.buf)) + 1):
            suf = self.buf[-k:]
            if any(s.startswith(suf) for s in self.stops):
                hold = k
        out, self.buf = (self.buf[:-hold], self.buf[-hold:]) if hold else (self.buf, "")
        return out, False

    def flush(self) -> str:
        out, self.buf = self.buf, ""
        return out


class Backend:
    def __init__(self, tokenizer: Tokenizer):
        self.tok = tokenizer

    async def generate(self, request: dict, context: Context,
                       engine: Callable[[dict, Context], AsyncIterator[dict]]) -> AsyncIterator[dict]:
        """request: PreprocessedRequest dict; yields BackendOutput dicts
        {token_ids, tokens, text, log_probs, cum_log_probs, finish_reason}."""
        sc = request.get("stop_conditions") or {}
        jail = StopJail(list(sc.get("stop") or []))
        ds = self.tok.decode_stream(request.get("token_ids") or [],
                                    skip_special_tokens=(request.get("output_options") or {}).get(
                                        "skip_special_tokens", True) is not False)
        cum = 0.0
        step = ds.step
        jailed = bool(jail.stops)
        async for out in engine(request, context):
            ids = out.get("token_ids") or []
            if len(ids) == 1:  # the common case: one token per engine step
                text = step(ids[0]) or ""
            else:
                text = "".join(p for p in map(step, ids) if p)
            lps = out.get("log_probs") or []
            if lps:
                cum += sum(lps)
            matched = False
            if jailed:
                text, matched = jail.push(text)
            fr = out.get("finish_reason")
            if matched:
                context.stop_generating()
                yield {"token_ids": ids, "text": text, "log_probs": lps, "cum_log_probs": cum, "finish_reason": "stop"}
                return
            if fr is not None:
                text += jail.flush()
            yield {"token_ids": ids, "text": text, "log_probs": lps, "cum_log_probs": cum, "finish_reason": fr}
            if fr is not None:
                return
