"""Engines behind the pipeline (reference lib/llm/src/engines.rs and
lib/engines/*):

* token level ("core", takes PreprocessedRequest, yields LLMEngineOutput):
    - `NativeEngine`       the first-party MI355X engine (`out=native`)
    - `EchoEngineCore`     echoes the prompt tokens (`out=echo_core`)
    - `PythonTokenEngine`  user file with `async def generate(request)` (`out=pytok:file.py`)
* OpenAI level ("full", takes a chat request dict, yields chat chunks):
    - `EchoEngineFull`     echoes the last user message (`out=echo_full`)
    - `PythonStringEngine` user file (`out=pystr:file.py`)

Echo delay: DYN_TOKEN_ECHO_DELAY_MS (default 10 ms, engines.rs:67).
"""
from __future__ import annotations

import asyncio
import importlib.util
import inspect
import os
import sys
import time
import uuid
from typing import AsyncIterator

from ..runtime.context import Context
from .protocols import ChatChunkChoice, ChatCompletionChunk, ChatDelta, new_request_id


def echo_delay() -> float:
    return float(os.environ.get("DYN_TOKEN_ECHO_DELAY_MS", "10")) / 1000.0


class EchoEngineCore:
    kind = "core"

    async def generate(self, request: dict, context: Context) -> AsyncIterator[dict]:
        delay = echo_delay()
        toks = list(request.get("token_ids") or [])
        mx = (request.get("stop_conditions") or {}).get("max_tokens")
        if mx:
            toks = toks[:mx]
        for i, t in enumerate(toks):
            if context.is_stopped():
                yield {"token_ids": [], "finish_reason": "cancelled"}
                return
            if delay:
                await asyncio.sleep(delay)
            yield {"token_ids": [t], "log_probs": [0.0],
                   "finish_reason": "stop" if i == len(toks) - 1 else None}
        if not toks:
            yield {"token_ids": [], "finish_reason": "stop"}


class EchoEngineFull:
    kind = "full"

    async def generate(self, request: dict, context: Context) -> AsyncIterator[dict]:
        delay = echo_delay()
        msgs = request.get("messages") or []
        text = ""
        for m in reversed(msgs):
            if m.get("role") == "user":
                c = m.get("content")
                text = c if isinstance(c, str) else "".join(p.get("text", "") for p in (c or []))
                break
        rid = new_request_id()
        model = request.get("model", "echo")
        first = True
        for i, ch in enumerate(text):
            if context.is_stopped():
                break
            if delay:
                await asyncio.sleep(delay)
            yield ChatCompletionChunk(id=rid, model=model, choices=[ChatChunkChoice(
                delta=ChatDelta(role="assistant" if first else None, content=ch))]).model_dump(exclude_none=True)
            first = False
        yield ChatCompletionChunk(id=rid, model=model, choices=[ChatChunkChoice(
            delta=ChatDelta(content=""), finish_reason="stop")]).model_dump(exclude_none=True)


class NativeEngine:
    """Token-level adapter over :class:`AsyncLLMEngine` (in-process)."""

    kind = "core"

    def __init__(self, async_engine, eos_token_ids: list[int] | None = None):
        self.ae = async_engine
        self.eos = eos_token_ids

    async def generate(self, request: dict, context: Context) -> AsyncIterator[dict]:
        from ..engine.request import SamplingParams

        params = SamplingParams.from_preprocessed(request, self.eos)
        rid = request.get("request_id") or context.id or uuid.uuid4().hex
        remote = bool(request.get("remote_prefill"))
        async for out in self.ae.generate(rid, request["token_ids"], params, context=context,
                                          remote_prefill=remote, remote_meta=request.get("remote_meta")):
            yield out


def _load_user_module(path: str, argv: list[str] | None = None):
    spec = importlib.util.spec_from_file_location(f"dx_user_engine_{abs(hash(path))}", path)
    mod = importlib.util.module_from_spec(spec)
    old = sys.argv
    sys.argv = [path] + list(argv or [])
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.argv = old
    if not hasattr(mod, "generate"):
        raise AttributeError(f"{path} must define `async def generate(request)`")
    return mod


class PythonTokenEngine:
    """`pytok:file.py` -- generate(PreprocessedRequest dict) yields LLMEngineOutput dicts
    (docs/guides/dynamo_run.md:355-378 ABI)."""

    kind = "core"

    def __init__(self, path: str, argv: list[str] | None = None):
        self.mod = _load_user_module(path, argv)

    async def generate(self, request: dict, context: Context) -> AsyncIterator[dict]:
        fn = self.mod.generate
        gen = fn(request, context) if len(inspect.signature(fn).parameters) >= 2 else fn(request)
        async for out in gen:
            if context.is_stopped():
                break
            yield out


class PythonStringEngine(PythonTokenEngine):
    """`pystr:file.py` -- generate(chat request dict) yields chat chunk dicts."""

    kind = "full"
