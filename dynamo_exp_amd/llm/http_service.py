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
from bisect import bisect_left
import logging
import time
from dataclasses import dataclass, field
from typing import Any

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse
from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

from ..runtime.context import Context
from ..utils.tracing import stage
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


def observe_many(hist, values: list[float]) -> None:
    """Histogram.observe for a batch: one bucket / sum update per bucket
    touched instead of per value (same result as observing one by one)."""
    if not values:
        return
    bounds, buckets, total = getattr(hist, "_upper_bounds", None), getattr(hist, "_buckets", None), \
        getattr(hist, "_sum", None)
    if bounds is None or buckets is None or total is None:
        for v in values:
            hist.observe(v)
        return
    counts: dict[int, int] = {}
    for v in values:
        i = bisect_left(bounds, v)
        counts[i] = counts.get(i, 0) + 1
    for i, c in counts.items():
        buckets[i].inc(c)
    total.inc(sum(values))


@dataclass
class Reply:
    status: int
    body: Any = None
    headers: dict = field(default_factory=dict)
    stream: Any = None  # async iterator of SSE event bytes


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
        self._mchildren: dict[str, tuple] = {}
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
        """The same routes as an ASGI app (in-process tests drive it through
        httpx.ASGITransport); `run()` serves them with the native asyncio
        HTTP/1.1 server (http_server.py) instead of uvicorn + Starlette."""
        app = FastAPI(title="dynamo_exp_amd OpenAI frontend")

        @app.get("/v1/models")
        async def models():
            return self.models_body()

        @app.get("/health")
        async def health():
            return self.health_body()

        @app.get("/live")
        async def live():
            return {"status": "live"}

        @app.get("/metrics")
        async def metrics():
            return PlainTextResponse(self.metrics_text(), media_type="text/plain; version=0.0.4")

        async def asgi_reply(request: Request, endpoint: str):
            r = await self.handle(endpoint, await request.body(), request.headers)
            if r.stream is None:
                return JSONResponse(r.body, r.status, headers=r.headers)
            return StreamingResponse(r.stream, media_type="text/event-stream", headers=r.headers)

        @app.post("/v1/chat/completions")
        async def chat(request: Request):
            return await asgi_reply(request, "chat_completions")

        @app.post("/v1/completions")
        async def completions(request: Request):
            return await asgi_reply(request, "completions")

        return app

    def models_body(self) -> dict:
        return ModelList(data=[ModelInfo(id=m) for m in self.manager.models()]).model_dump()

    def health_body(self) -> dict:
        return {"status": "healthy", "models": self.manager.models()}

    def metrics_text(self) -> str:
        return generate_latest(self.metrics.registry).decode()

    def _children(self, model: str) -> tuple:
        """Per-model labelled metric children, resolved once (labels() per
        streamed chunk was a measurable share of the frontend's CPU)."""
        c = self._mchildren.get(model)
        if c is None:
            m = self.metrics
            c = self._mchildren[model] = (m.ttft.labels(model), m.itl.labels(model), m.output_tokens.labels(model),
                                          m.inflight.labels(model), m.duration.labels(model))
        return c

    async def handle(self, endpoint: str, raw: bytes, headers) -> "Reply":
        """One OpenAI request, transport-agnostic: a unary JSON reply or an
        SSE byte stream (reference lib/llm/src/http/service/openai.rs:222-321)."""
        try:
            body = json.loads(raw)
            if not isinstance(body, dict):
                raise ValueError("not an object")
        except Exception:
            return Reply(400, {"error": {"message": "invalid JSON", "type": "invalid_request_error"}})
        self._apply_template(body)
        try:
            req = ChatCompletionRequest(**body) if endpoint == "chat_completions" else CompletionRequest(**body)
        except Exception as e:
            return Reply(400, {"error": {"message": str(e), "type": "invalid_request_error"}})
        table = self.manager.chat if endpoint == "chat_completions" else self.manager.completion
        eng = table.get(req.model)
        streaming = bool(req.stream)
        rtype = "stream" if streaming else "unary"
        m = self.metrics
        if eng is None:
            m.requests.labels(req.model, endpoint, rtype, "error").inc()
            return Reply(404, {"error": {"message": f"model {req.model} not found", "type": "not_found"}})
        # honour a caller-supplied x-request-id (tracing across services) and echo it back
        rid = headers.get("x-request-id") or new_request_id()
        ctx = Context(rid)
        stage("http.recv", rid)
        gen = eng.chat(req, ctx) if endpoint == "chat_completions" else eng.completion(req, ctx)
        t0 = time.perf_counter()
        ttft, itl, chunks, inflight, duration = self._children(req.model)
        inflight.inc()

        async def timed(stream):
            # per-chunk gaps are batched into the histogram every 32 chunks
            # (one prometheus observe + counter inc per chunk were ~10 % of
            # the frontend's CPU at node scale)
            last = None
            gaps: list[float] = []
            n = 0
            try:
                async for ch in stream:
                    now = time.perf_counter()
                    if last is None:
                        ttft.observe(now - t0)
                        stage("http.first", rid, now)
                    else:
                        gaps.append(now - last)
                        if len(gaps) >= 32:
                            observe_many(itl, gaps)
                            gaps = []
                    last = now
                    n += 1
                    yield ch
            finally:
                observe_many(itl, gaps)
                chunks.inc(n)
                inflight.dec()
                duration.observe(time.perf_counter() - t0)

        if not streaming:
            try:
                agg = aggregate_chat if endpoint == "chat_completions" else aggregate_completion
                resp = await agg(timed(gen))
                m.requests.labels(req.model, endpoint, rtype, "success").inc()
                return Reply(200, resp, {"x-request-id": rid})
            except Exception as e:
                log.exception("request failed")
                m.requests.labels(req.model, endpoint, rtype, "error").inc()
                return Reply(500, {"error": {"message": str(e), "type": "internal_error"}})

        dumps = json.dumps

        async def sse():
            status = "success"
            try:
                async for ch in timed(gen):
                    if "event" in ch and "choices" not in ch:
                        yield f"event: {ch['event']}\ndata: {dumps(ch.get('comment'))}\n\n".encode()
                        continue
                    yield b"data: " + dumps(ch).encode() + b"\n\n"
                yield b"data: [DONE]\n\n"
            except (asyncio.CancelledError, GeneratorExit):
                status = "cancelled"
                ctx.stop_generating()  # client went away
                raise
            except Exception as e:
                status = "error"
                log.exception("stream failed")
                yield f"event: error\ndata: {dumps({'message': str(e)})}\n\n".encode()
            finally:
                m.requests.labels(req.model, endpoint, rtype, status).inc()

        return Reply(200, None, {"x-request-id": rid}, sse())

    # ------------------------------------------------------------------ run
    async def run(self) -> None:
        from .http_server import serve_http

        srv = await serve_http(self, self.host, self.port, reuse_port=self.reuse_port)
        if not self.port:
            self.port = srv.servers[0].sockets[0].getsockname()[1]
        self._server = srv
        await srv.serve_forever()

    async def start_background(self) -> asyncio.Task:
        t = asyncio.create_task(self.run())
        while self._server is None:
            await asyncio.sleep(0.02)
            if t.done():
                t.result()
        return t

    def stop(self) -> None:
        if self._server is not None:
            self._server.close()
