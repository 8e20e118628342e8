"""Server-sent-events client codec: turn an OpenAI SSE byte stream back into
typed chunks and fold them into one unary response.

Behaviour of the reference's `SseLineCodec` + `from_sse_stream`
(lib/llm/src/protocols/codec.rs, lib/llm/src/protocols/openai/*/aggregator.rs):

* a message ends at a blank line; `data:` lines of one message are joined
  with newlines (a JSON object may be split over several `data:` lines);
* `:` lines are comments, collected per message; `event:`, `id:` set the
  message's event type and id; `retry:` and unknown fields are ignored;
* `data: [DONE]` contributes nothing (the end-of-stream marker);
* `event: error` turns the message into an error (its comments are the text);
* a `data` payload that does not deserialize into the response chunk type is
  an error for the whole fold.

Used by the HTTP client paths (tools/loadgen.py) and by the parity tests that
replay the reference's recorded streams (tests/test_parity_fixtures.py).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Iterable, Iterator

from pydantic import ValidationError

from .protocols import ChatCompletionChunk, CompletionResponse


class SseDecodeError(ValueError):
    pass


@dataclass
class SseMessage:
    id: str | None = None
    event: str | None = None
    data: str | None = None
    comments: list[str] = field(default_factory=list)

    def json(self):
        if self.data is None:
            raise SseDecodeError("no data: message to decode")
        try:
            return json.loads(self.data)
        except json.JSONDecodeError as e:
            raise SseDecodeError(f"failed to deserialize data: {e}") from e


def parse_sse(text: str | Iterable[str]) -> Iterator[SseMessage]:
    """Messages of an SSE stream (a whole string or an iterable of lines)."""
    lines = text.splitlines() if isinstance(text, str) else (l.rstrip("\r\n") for l in text)
    data: list[str] = []
    ev = mid = None
    comments: list[str] = []
    for line in lines:
        line = line.rstrip("\r\n")
        if not line:
            if data or ev is not None or mid is not None or comments:
                yield SseMessage(mid, ev, "\n".join(data) if data else None, comments)
                data, ev, mid, comments = [], None, None, []
            continue
        if line.startswith(":"):
            comments.append(line[1:].strip())
            continue
        name, sep, value = line.partition(":")
        value = value.lstrip(" ") if sep else ""
        if name == "data":
            if value != "[DONE]":
                data.append(value)
        elif name == "event":
            ev = value
        elif name == "id":
            if "\0" not in value:
                mid = value
    if data or ev is not None or mid is not None or comments:
        yield SseMessage(mid, ev, "\n".join(data) if data else None, comments)


def _chunks(messages: Iterable[SseMessage], model):
    for m in messages:
        if m.event == "error":
            raise SseDecodeError("\n".join(m.comments) or "`event: error` detected, but no error message found")
        if m.data is None:
            continue  # comment / keep-alive only
        try:
            yield model.model_validate(m.json())
        except ValidationError as e:
            raise SseDecodeError(f"failed to deserialize data: {e.errors()[0]['msg']}") from e


def chat_from_sse(messages: Iterable[SseMessage]) -> dict:
    """Fold chat.completion.chunk messages into a chat.completion (per choice
    index: role, concatenated content, last finish reason)."""
    rid = model = created = None
    usage = None
    choices: dict[int, dict] = {}
    for ch in _chunks(messages, ChatCompletionChunk):
        rid, model, created = ch.id, ch.model, ch.created
        if ch.usage is not None:
            usage = ch.usage.model_dump()
        for c in ch.choices:
            st = choices.setdefault(c.index, {"role": "assistant", "content": [], "finish_reason": None})
            if c.delta.role:
                st["role"] = c.delta.role
            if c.delta.content:
                st["content"].append(c.delta.content)
            if c.finish_reason:
                st["finish_reason"] = c.finish_reason
    if rid is None:
        raise SseDecodeError("empty stream")
    out = {"id": rid, "object": "chat.completion", "created": created, "model": model,
           "choices": [{"index": i, "message": {"role": st["role"], "content": "".join(st["content"])},
                        "finish_reason": st["finish_reason"]} for i, st in sorted(choices.items())]}
    if usage is not None:
        out["usage"] = usage
    return out


def completion_from_sse(messages: Iterable[SseMessage]) -> dict:
    """Fold text_completion chunks into one text_completion."""
    rid = model = created = None
    usage = None
    choices: dict[int, dict] = {}
    for ch in _chunks(messages, CompletionResponse):
        rid, model, created = ch.id, ch.model, ch.created
        if ch.usage is not None:
            usage = ch.usage.model_dump()
        for c in ch.choices:
            st = choices.setdefault(c.index, {"text": [], "finish_reason": None})
            st["text"].append(c.text or "")
            if c.finish_reason:
                st["finish_reason"] = c.finish_reason
    if rid is None:
        raise SseDecodeError("empty stream")
    out = {"id": rid, "object": "text_completion", "created": created, "model": model,
           "choices": [{"index": i, "text": "".join(st["text"]), "finish_reason": st["finish_reason"]}
                       for i, st in sorted(choices.items())]}
    if usage is not None:
        out["usage"] = usage
    return out
