"""OpenAI-compatible HTTP frontend (reference lib/llm/src/http/service/*).

Routes: POST /v1/chat/completions, POST /v1/completions, GET /v1/models,
GET /metrics (Prometheus), GET /health, GET /live.

* requests are always streamed internally and folded when `stream=false`
  (openai.rs:222-321); SSE ends with `data: [DONE]`;
* a client disconnect stops generation upstream (Context.stop_generating,
  openai.rs:433-466);
* optional request template supplies default model / temperature / max_tokens
  (request_template.rs);
* metrics: `{prefix}_http_service_requests_total{model,endpoint,request_type,status}`,
  `_inflight_requests{model}`, `_request_duration_seconds{model}` (metrics.rs:92-133)
  plus TTFT / inter-token-latency histograms and output-token counters, which
  the reference lacks.
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from dataclasses import dataclass
from typing import Any

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse
from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

from ..runtime.context import Context
from .preprocessor import aggregate_chat, aggregate_completion
from .protocols import ChatCompletionRequest, CompletionRequest, ModelInfo, ModelList, new_request_id

log = logging.getLogger("dynamo_exp_amd.http")


@dataclass
class RequestTemplate:
    model: str | None = None
    temperature: float | None = None
    max_completion_tokens: int | None = None

    @classmethod
    def load(cls, path: str) -> "RequestTemplate":
        with open(path) as f:
            d = json.load(f)
        return cls(d.get("model"), d.get("temperature"), d.get("max_completion_tokens") or d.get("max_tokens"))


class Metrics:
    def __init__(self, prefix: str = "dynamo"):
        self.registry = CollectorRegistry()
        p = f"{prefix}_http_service"
        self.requests = Counter(f"{p}_requests_total", "requests", ["model", "endpoint", "request_type", "status"],
                                registry=self.registry)
        self.inflight = Gauge(f"{p}_inflight_requests", "inflight", ["model"], registry=self.registry)
        buckets = [0, 1, 2, 4, 8, 16, 32, 64, 128, 256]
        self.duration = Histogram(f"{p}_request_duration_seconds", "duration", ["model"], buckets=buckets,
                                  registry=self.registry)
        self.ttft = Histogram(f"{p}_time_to_first_token_seconds", "TTFT", ["model"],
                              buckets=[.005, .01, .025, .05, .1, .25, .5, 1, 2.5, 5, 10, 30], registry=self.registry)
        self.itl = Histogram(f"{p}_inter_token_latency_seconds", "ITL", ["model"],
                             buckets=[.001, .0025, .005, .01, .02, .04, .08, .16, .32, 1], registry=self.registry)
        self.output_tokens = Counter(f"{p}_output_chunks_total", "streamed chunks", ["model"], registry=self.registry)


class ModelManager:
    def __init__(self):
        self.chat: dict[str, Any] = {}
        self.completion: dict[str, Any] = {}

    def add_chat_model(self, name: str, engine) -> None:
        self.chat[name] = engine

    def add_completion_model(self, name: str, engine) -> None:
        self.completion[name] = engine

    def remove_model(self, name: str) -> None:
        self.chat.pop(name, None)
        self.completion.pop(name, None)

    def remove_chat_model(self, name: str) -> None:
        self.chat.pop(name, None)

    def remove_completion_model(self, name: str) -> None:
        self.completion.pop(name, None)

    def models(self) -> list[str]:
        return sorted(set(self.chat) | set(self.completion))


class HttpService:
    def __init__(self, host: str = "0.0.0.0", port: int = 8080, request_template: RequestTemplate | None = None,
                 metrics_prefix: str = "dynamo", reuse_port: bool = False):
        self.host, self.port = host, port
        # reuse_port: several frontend processes share the port (SO_REUSEPORT,
        # the kernel spreads connections over them) -- one Python process per
        # core instead of one event loop carrying every SSE stream of the node
        self.reuse_port = reuse_port
        self.manager = ModelManager()
        self.template = request_template
        self.metrics = Metrics(metrics_prefix)
        self.app = self._build()
        self._server = None

    # ------------------------------------------------------------------ app
    def _apply_template(self, body: dict) -> None:
        t = self.template
        if t is None:
            return
        if not body.get("model") and t.model:
            body["model"] = t.model
        if body.get("temperature") is None and t.temperature is not None:
            body["temperature"] = t.temperature
        if body.get("max_tokens") is None and body.get("max_completion_tokens") is None and t.max_completion_tokens:
            body["max_completion_tokens"] = t.max_completion_tokens

    def _build(self) -> FastAPI:
        app = FastAPI(title="dynamo_exp_amd OpenAI frontend")

        @app.get("/v1/models")
        async def models():
            return ModelList(data=[ModelInfo(id=m) for m in self.manager.models()]).model_dump()

        @app.get("/health")
        async def health():
            return {"status": "healthy", "models": self.manager.models()}

        @app.get("/live")
        async def live():
            return {"status": "live"}

        @app.get("/metrics")
        async def metrics():
            return PlainTextResponse(generate_latest(self.metrics.registry).decode(),
                                     media_type="text/plain; version=0.0.4")

        @app.post("/v1/chat/completions")
        async def chat(request: Request):
            return await self._handle(request, "chat_completions")

        @app.post("/v1/completions")
        async def completions(request: Request):
            return await self._handle(request, "completions")

        return app

    async def _handle(self, request: Request, endpoint: str):
        try:
            body = await request.json()
        except Exception:
            return JSONResponse({"error": {"message": "invalid JSON", "type": "invalid_request_error"}}, 400)
        self._apply_template(body)
        try:
            req = ChatCompletionRequest(**body) if endpoint == "chat_completions" else CompletionRequest(**body)
        except Exception as e:
            return JSONResponse({"error": {"message": str(e), "type": "invalid_request_error"}}, 400)
        table = self.manager.chat if endpoint == "chat_completions" else self.manager.completion
        eng = table.get(req.model)
        streaming = bool(req.stream)
        rtype = "stream" if streaming else "unary"
        m = self.metrics
        if eng is None:
            m.requests.labels(req.model, endpoint, rtype, "error").inc()
            return JSONResponse({"error": {"message": f"model {req.model} not found", "type": "not_found"}}, 404)
        # honour a caller-supplied x-request-id (tracing across services) and echo it back
        rid = request.headers.get("x-request-id") or new_request_id()
        ctx = Context(rid)
        gen = eng.chat(req, ctx) if endpoint == "chat_completions" else eng.completion(req, ctx)
        t0 = time.perf_counter()
        m.inflight.labels(req.model).inc()

        async def timed(stream):
            last = None
            try:
                async for ch in stream:
                    now = time.perf_counter()
                    if last is None:
                        m.ttft.labels(req.model).observe(now - t0)
                    else:
                        m.itl.labels(req.model).observe(now - last)
                    last = now
                    m.output_tokens.labels(req.model).inc()
                    yield ch
            finally:
                m.inflight.labels(req.model).dec()
                m.duration.labels(req.model).observe(time.perf_counter() - t0)

        if not streaming:
            try:
                agg = aggregate_chat if endpoint == "chat_completions" else aggregate_completion
                resp = await agg(timed(gen))
                m.requests.labels(req.model, endpoint, rtype, "success").inc()
                return JSONResponse(resp, headers={"x-request-id": rid})
            except Exception as e:
                log.exception("request failed")
                m.requests.labels(req.model, endpoint, rtype, "error").inc()
                return JSONResponse({"error": {"message": str(e), "type": "internal_error"}}, 500)

        async def sse():
            status = "success"
            try:
                async for ch in timed(gen):
                    if "event" in ch and "choices" not in ch:
                        yield f"event: {ch['event']}\ndata: {json.dumps(ch.get('comment'))}\n\n"
                        continue
                    yield f"data: {json.dumps(ch)}\n\n"
                yield "data: [DONE]\n\n"
            except (asyncio.CancelledError, GeneratorExit):
                status = "cancelled"
                ctx.stop_generating()  # client went away
                raise
            except Exception as e:
                status = "error"
                log.exception("stream failed")
                yield f"event: error\ndata: {json.dumps({'message': str(e)})}\n\n"
            finally:
                m.requests.labels(req.model, endpoint, rtype, status).inc()

        return StreamingResponse(sse(), media_type="text/event-stream", headers={"x-request-id": rid})

    # ------------------------------------------------------------------ run
    async def run(self) -> None:
        import uvicorn

        cfg = uvicorn.Config(self.app, host=self.host, port=self.port, log_level="warning", loop="asyncio",
                             timeout_keep_alive=30, backlog=4096)
        self._server = uvicorn.Server(cfg)
        socks = None
        if self.reuse_port:
            import socket

            sock = socket.socket(socket.AF_INET6 if ":" in self.host else socket.AF_INET, socket.SOCK_STREAM)
            sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
            sock.bind((self.host, self.port))
            sock.set_inheritable(True)
            socks = [sock]
        await self._server.serve(sockets=socks)

    async def start_background(self) -> asyncio.Task:
        t = asyncio.create_task(self.run())
        while self._server is None or not self._server.started:
            await asyncio.sleep(0.02)
            if t.done():
                t.result()
        return t

    def stop(self) -> None:
        if self._server is not None:
            self._server.should_exit = True
