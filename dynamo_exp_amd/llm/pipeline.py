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

import logging
from typing import AsyncIterator

from ..runtime.context import Context
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
    """Routes PreprocessedRequests to instances of a worker endpoint."""

    def __init__(self, client, mode: str = "round_robin", kv_router=None):
        self.client, self.mode, self.kv = client, mode, kv_router

    async def generate(self, request: dict, ctx: Context) -> AsyncIterator[dict]:
        if self.mode == "kv" and self.kv is not None:
            wid, overlap = await self.kv.schedule(request["token_ids"], self.client.instance_ids())
            request["estimated_prefix_hit_num_blocks"] = overlap
            stream = await self.client.direct(request, wid, ctx)
            try:
                async for out in stream:
                    yield out
            finally:
                self.kv.release(wid)
            return
        if self.mode == "random":
            stream = await self.client.random(request, ctx)
        else:
            stream = await self.client.round_robin(request, ctx)
        async for out in stream:
            yield out


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

    async def chat(self, req, ctx):
        async for ch in self.router.generate(req.model_dump(exclude_none=True), ctx):
            yield ch

    async def completion(self, req, ctx):
        async for ch in self.router.generate(req.model_dump(exclude_none=True), ctx):
            yield ch


def core_handler(backend: Backend, engine):
    """Worker-side endpoint handler: PreprocessedRequest -> BackendOutput stream."""

    async def handler(request: dict, ctx: Context):
        async for out in backend.generate(request, ctx, engine.generate):
            yield out

    return handler


async def serve_core_engine(endpoint, backend: Backend, engine, stats_handler=None) -> None:
    await endpoint.serve_endpoint(core_handler(backend, engine), stats_handler=stats_handler)
