"""Serving pipelines (reference lib/runtime pipeline graph):
plain composition of async generators.

frontend side (OpenAI in, OpenAI chunks out):
  LocalPipeline    preprocess -> Backend(detok/stop) -> token engine (in-process)
  RemotePipeline   preprocess -> WorkerRouter (random | round_robin | kv) ->
                   [worker: Backend -> token engine] -> chunks
  FullPipeline     OpenAI-level engine (echo_full / pystr) as is
  ChatForwarder    raw OpenAI request -> a `chat`-type endpoint (e.g. a Processor component)
worker side:
  serve_core_engine(endpoint, backend, engine)  registers Backend+engine as an endpoint handler
"""
from __future__ import annotations

import asyncio
import logging
import random
from typing import AsyncIterator

from ..runtime.context import Context
from ..runtime.transport import EndpointError
from .backend import Backend
from .preprocessor import OpenAIPreprocessor
from .protocols import ChatCompletionRequest, CompletionRequest

log = logging.getLogger("dynamo_exp_amd.pipeline")


class LocalPipeline:
    def __init__(self, preproc: OpenAIPreprocessor, backend: Backend, engine):
        self.pre, self.backend, self.engine = preproc, backend, engine

    async def chat(self, req: ChatCompletionRequest, ctx: Context) -> AsyncIterator[dict]:
        pre, ann = self.pre.preprocess_chat(req)
        d = pre.model_dump()
        d["request_id"] = ctx.id
        stream = self.backend.generate(d, ctx, self.engine.generate)
        async for ch in self.pre.chat_stream(req, stream, ann, ctx.id):
            yield ch

    async def completion(self, req: CompletionRequest, ctx: Context) -> AsyncIterator[dict]:
        pre, ann = self.pre.preprocess_completion(req)
        d = pre.model_dump()
        d["request_id"] = ctx.id
        stream = self.backend.generate(d, ctx, self.engine.generate)
        async for ch in self.pre.completion_stream(req, stream, ann, ctx.id):
            yield ch


class WorkerRouter:
    """Routes PreprocessedRequests to instances of a worker endpoint.

    Retry-before-first-token: if the chosen worker fails before
    it produced anything (dead instance, connection refused, error prologue),
    the request is re-routed to another instance, up to `retries` times;
    once output has streamed, a failure ends the stream as in the reference.
    """

    def __init__(self, client, mode: str = "round_robin", kv_router=None, retries: int = 2):
        self.client, self.mode, self.kv = client, mode, kv_router
        self.retries = retries
        self._rr = 0

    async def _open(self, request: dict, ctx: Context, exclude: set):
        ids = [i for i in self.client.instance_ids() if i not in exclude] or self.client.instance_ids()
        if not ids:
            raise EndpointError(f"no instances for {self.client.endpoint.path}")
        if self.mode == "kv" and self.kv is not None:
            wid, overlap = await self.kv.schedule(request["token_ids"], ids)
            request["estimated_prefix_hit_num_blocks"] = overlap
        elif self.mode == "random":
            wid = random.choice(ids)
        else:
            wid = ids[self._rr % len(ids)]
            self._rr += 1
        return wid, await self.client.direct(request, wid, ctx)

    async def generate(self, request: dict, ctx: Context) -> AsyncIterator[dict]:
        tried: set = set()
        for attempt in range(self.retries + 1):
            wid = None
            started = False
            try:
                wid, stream = await self._open(request, ctx, tried)
                async for out in stream:
                    started = True
                    yield out
                return
            except (ConnectionError, OSError, asyncio.TimeoutError, EndpointError) as e:
                if started or attempt == self.retries or ctx.is_stopped():
                    raise
                log.warning("worker %s failed before first token (%s); re-routing", wid, e)
                if wid is not None:
                    tried.add(wid)
            finally:
                if self.kv is not None and wid is not None and self.mode == "kv":
                    self.kv.release(wid)


class RemotePipeline(LocalPipeline):
    def __init__(self, preproc: OpenAIPreprocessor, router: WorkerRouter):
        self.pre = preproc
        self.router = router

    async def chat(self, req, ctx):
        pre, ann = self.pre.preprocess_chat(req)
        d = pre.model_dump()
        d["request_id"] = ctx.id
        async for ch in self.pre.chat_stream(req, self.router.generate(d, ctx), ann, ctx.id):
            yield ch

    async def completion(self, req, ctx):
        pre, ann = self.pre.preprocess_completion(req)
        d = pre.model_dump()
        d["request_id"] = ctx.id
        async for ch in self.pre.completion_stream(req, self.router.generate(d, ctx), ann, ctx.id):
            yield ch


class FullPipeline:
    def __init__(self, engine):
        self.engine = engine

    async def chat(self, req: ChatCompletionRequest, ctx: Context) -> AsyncIterator[dict]:
        async for ch in self.engine.generate(req.model_dump(exclude_none=True), ctx):
            yield ch

    async def completion(self, req: CompletionRequest, ctx: Context) -> AsyncIterator[dict]:
        d = req.model_dump(exclude_none=True)
        d["messages"] = [{"role": "user", "content": req.prompt if isinstance(req.prompt, str) else str(req.prompt)}]
        async for ch in self.engine.generate(d, ctx):
            # convert chat chunk -> completion chunk
            yield {"id": ch.get("id"), "object": "text_completion", "created": ch.get("created"),
                   "model": ch.get("model"),
                   "choices": [{"index": 0, "text": c.get("delta", {}).get("content") or "",
                                "finish_reason": c.get("finish_reason")} for c in ch.get("choices", [])]}


class ChatForwarder:
    """ModelType chat/completion entries: forward the raw OpenAI request to a
    worker endpoint that already speaks OpenAI (reference discovery.rs:314)."""

    def __init__(self, client, mode: str = "round_robin"):
        self.router = WorkerRouter(client, mode)

    def chat(self, req, ctx):  # the router's stream itself: no extra async hop per chunk
        return self.router.generate(req.model_dump(exclude_none=True), ctx)

    def completion(self, req, ctx):
        return self.router.generate(req.model_dump(exclude_none=True), ctx)


def core_handler(backend: Backend, engine):
    """Worker-side endpoint handler: PreprocessedRequest -> BackendOutput stream."""

    async def handler(request: dict, ctx: Context):
        async for out in backend.generate(request, ctx, engine.generate):
            yield out

    return handler


async def serve_core_engine(endpoint, backend: Backend, engine, stats_handler=None) -> None:
    await endpoint.serve_endpoint(core_handler(backend, engine), stats_handler=stats_handler)
