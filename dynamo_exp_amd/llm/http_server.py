"""Native asyncio HTTP/1.1 server for the OpenAI frontend.

The reference frontend is a multi-threaded axum server whose per-token path is
compiled Rust (lib/llm/src/http/service/openai.rs:222-321, service_v2.rs).
Behind uvicorn + Starlette + h11 every streamed chunk cost ~50 us of pure
Python in this frontend (ASGI message dicts, h11 state machine, three wrapper
coroutines per send), so at node scale (2048 SSE streams x 13 tok/s) the
frontend, not the GPUs, set the latency.  This server speaks just enough
HTTP/1.1 for the OpenAI API on an `asyncio.Protocol`:

* request head parsed once per request (request line + headers, Content-Length
  or chunked body, `Expect: 100-continue`), keep-alive and pipelining (one
  request at a time per connection, in order), idle timeout;
* SSE streams go out as chunked transfer-encoding with ONE `transport.write`
  per event -- no per-chunk objects beyond the bytes themselves;
* flow control via `pause_writing` / `resume_writing` (a slow client stops its
  own stream only), client disconnect cancels the stream task, which stops
  generation upstream (`Context.stop_generating`);
* SO_REUSEPORT so several frontend processes share one port.

Routes and semantics are the ones of HttpService (the FastAPI app serves the
same handlers for in-process tests).
"""
from __future__ import annotations

import asyncio
import json
import logging
import socket
from collections import deque

log = logging.getLogger("dynamo_exp_amd.http")

_REASON = {100: "Continue", 200: "OK", 400: "Bad Request", 404: "Not Found", 405: "Method Not Allowed",
           411: "Length Required", 413: "Payload Too Large", 431: "Request Header Fields Too Large",
           500: "Internal Server Error", 501: "Not Implemented"}
MAX_HEAD = 64 << 10
MAX_BODY = 256 << 20
IDLE_TIMEOUT_S = 30.0
MAX_PIPELINED = 64  # queued requests per connection before reading pauses


class _Req:
    __slots__ = ("method", "path", "headers", "body", "keep_alive")

    def __init__(self, method, path, headers, body, keep_alive):
        self.method, self.path, self.headers, self.body, self.keep_alive = method, path, headers, body, keep_alive


class _BadRequest(Exception):
    def __init__(self, status: int, msg: str):
        super().__init__(msg)
        self.status = status


def _parse_chunked(buf: bytearray, start: int) -> tuple[bytes, int] | None:
    """Decode a chunked body starting at buf[start]; None if incomplete."""
    out = bytearray()
    i = start
    while True:
        j = buf.find(b"\r\n", i)
        if j < 0:
            return None
        try:
            n = int(bytes(buf[i:j]).split(b";", 1)[0].strip(), 16)
        except ValueError:
            raise _BadRequest(400, "bad chunk size")
        i = j + 2
        if n < 0 or len(out) + n > MAX_BODY:  # refuse on the declared size, before buffering the chunk
            raise _BadRequest(413, "body too large")
        if n == 0:
            k = buf.find(b"\r\n\r\n", i - 2)  # trailers (usually none) end with an empty line
            if k < 0:
                return None
            return bytes(out), k + 4
        if len(buf) < i + n + 2:
            return None
        out += buf[i:i + n]
        i += n + 2


class HttpProtocol(asyncio.Protocol):
    def __init__(self, svc):
        self.svc = svc
        self.buf = bytearray()
        self.transport = None
        self.task: asyncio.Task | None = None
        self.pending: deque = deque()
        self.paused = False
        self.waiter: asyncio.Future | None = None
        self.closed = False
        self.continued = False
        self.idle = None
        self.reading_paused = False

    # -------------------------------------------------------------- asyncio
    def connection_made(self, transport):
        self.transport = transport
        sock = transport.get_extra_info("socket")
        if sock is not None:
            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        self._arm_idle()

    def data_received(self, data):
        self.buf += data
        self._parse()

    def connection_lost(self, exc):
        self.closed = True
        if self.idle is not None:
            self.idle.cancel()
        if self.task is not None and not self.task.done():
            self.task.cancel()  # a streaming reply stops generation upstream
        self._wake()

    def pause_writing(self):
        self.paused = True

    def resume_writing(self):
        self.paused = False
        self._wake()

    def _wake(self):
        w, self.waiter = self.waiter, None
        if w is not None and not w.done():
            w.set_result(None)

    async def _drain(self):
        if self.paused and not self.closed:
            self.waiter = asyncio.get_running_loop().create_future()
            await self.waiter
        if self.closed:
            raise ConnectionResetError("client went away")

    def _arm_idle(self):
        if self.idle is not None:
            self.idle.cancel()
        self.idle = asyncio.get_running_loop().call_later(IDLE_TIMEOUT_S, self._idle_close)

    def _idle_close(self):
        if self.task is None and not self.pending and self.transport is not None:
            self.transport.close()

    # -------------------------------------------------------------- parsing
    def _parse(self):
        while not self.closed:
            try:
                req = self._take_request()
            except _BadRequest as e:
                self._write_simple(e.status, {"error": {"message": str(e), "type": "invalid_request_error"}},
                                   keep_alive=False)
                self.buf.clear()
                self.transport.close()
                return
            if req is None:
                return
            self.pending.append(req)
            if len(self.pending) >= MAX_PIPELINED and not self.reading_paused:
                self.reading_paused = True  # a client pipelining without reading: stop reading it
                self.transport.pause_reading()
            self._next()

    def _take_request(self) -> _Req | None:
        buf = self.buf
        end = buf.find(b"\r\n\r\n")
        if end < 0:
            if len(buf) > MAX_HEAD:
                raise _BadRequest(431, "request head too large")
            return None
        head = bytes(buf[:end]).decode("latin-1")
        lines = head.split("\r\n")
        parts = lines[0].split(" ")
        if len(parts) != 3 or not parts[2].startswith("HTTP/1."):
            raise _BadRequest(400, "bad request line")
        method, target, version = parts
        headers = {}
        for ln in lines[1:]:
            k, sep, v = ln.partition(":")
            if not sep:
                raise _BadRequest(400, "bad header line")
            headers[k.strip().lower()] = v.strip()
        conn = headers.get("connection", "").lower()
        keep_alive = ("close" not in conn) if version == "HTTP/1.1" else ("keep-alive" in conn)
        start = end + 4
        if "chunked" in headers.get("transfer-encoding", "").lower():
            got = _parse_chunked(buf, start)
            if got is None:
                self._maybe_continue(headers)
                return None
            body, used = got
        else:
            try:
                n = int(headers.get("content-length", "0"))
            except ValueError:
                raise _BadRequest(400, "bad content-length")
            if n < 0 or n > MAX_BODY:
                raise _BadRequest(413, "body too large")
            if len(buf) < start + n:
                self._maybe_continue(headers)
                return None
            body, used = bytes(buf[start:start + n]), start + n
        del buf[:used]
        self.continued = False
        return _Req(method, target.split("?", 1)[0], headers, body, keep_alive)

    def _maybe_continue(self, headers):
        if not self.continued and headers.get("expect", "").lower() == "100-continue" and self.task is None \
                and not self.pending:
            self.continued = True
            self.transport.write(b"HTTP/1.1 100 Continue\r\n\r\n")

    # -------------------------------------------------------------- serving
    def _next(self):
        if self.task is not None or not self.pending or self.closed:
            return
        if self.idle is not None:
            self.idle.cancel()
            self.idle = None
        req = self.pending.popleft()
        if self.reading_paused and len(self.pending) < MAX_PIPELINED // 2:
            self.reading_paused = False
            self.transport.resume_reading()
        self.task = asyncio.get_running_loop().create_task(self._serve(req))
        self.task.add_done_callback(self._done)

    def _done(self, t: asyncio.Task):
        self.task = None
        exc = None if t.cancelled() else t.exception()
        if exc is not None and not isinstance(exc, ConnectionError):
            log.error("http handler failed", exc_info=exc)
        if exc is not None and not self.closed:
            # the reply may be half written (a chunked SSE head without its
            # terminator): the connection cannot carry another response
            self.closed = True
            self.transport.close()
            return
        if self.closed:
            return
        if self.pending:
            self._next()
        else:
            self._arm_idle()

    def _head(self, status: int, ctype: str, extra: dict, keep_alive: bool, length: int | None) -> bytes:
        h = [f"HTTP/1.1 {status} {_REASON.get(status, 'Unknown')}", f"content-type: {ctype}"]
        h.append(f"content-length: {length}" if length is not None else "transfer-encoding: chunked")
        for k, v in extra.items():
            h.append(f"{k}: {v}")
        if not keep_alive:
            h.append("connection: close")
        return ("\r\n".join(h) + "\r\n\r\n").encode("latin-1")

    def _write_simple(self, status: int, obj, keep_alive: bool, extra: dict | None = None,
                      ctype: str = "application/json") -> None:
        body = obj if isinstance(obj, bytes) else json.dumps(obj).encode()
        self.transport.write(self._head(status, ctype, extra or {}, keep_alive, len(body)) + body)
        if not keep_alive:
            self.transport.close()

    async def _serve(self, req: _Req) -> None:
        svc, ka = self.svc, req.keep_alive
        route = (req.method, req.path)
        if route == ("POST", "/v1/chat/completions") or route == ("POST", "/v1/completions"):
            ep = "chat_completions" if req.path == "/v1/chat/completions" else "completions"
            r = await svc.handle(ep, req.body, req.headers)
            if self.closed:
                if r.stream is not None:
                    await r.stream.aclose()
                return
            if r.stream is None:
                return self._write_simple(r.status, r.body, ka, r.headers)
            await self._stream(r, ka)
        elif route == ("GET", "/v1/models"):
            self._write_simple(200, svc.models_body(), ka)
        elif route == ("GET", "/health"):
            self._write_simple(200, svc.health_body(), ka)
        elif route == ("GET", "/live"):
            self._write_simple(200, {"status": "live"}, ka)
        elif route == ("GET", "/metrics"):
            self._write_simple(200, svc.metrics_text().encode(), ka, ctype="text/plain; version=0.0.4")
        elif req.path in ("/v1/chat/completions", "/v1/completions", "/v1/models", "/health", "/live", "/metrics"):
            self._write_simple(405, {"detail": "Method Not Allowed"}, ka)
        else:
            self._write_simple(404, {"detail": "Not Found"}, ka)

    async def _stream(self, r, keep_alive: bool) -> None:
        t = self.transport
        t.write(self._head(r.status, "text/event-stream; charset=utf-8",
                           dict(r.headers, **{"cache-control": "no-cache"}), keep_alive, None))
        stream = r.stream
        try:
            async for ev in stream:
                t.write(b"%x\r\n%b\r\n" % (len(ev), ev))
                if self.paused or self.closed:
                    await self._drain()
            t.write(b"0\r\n\r\n")
        finally:
            await stream.aclose()
        if not keep_alive:
            t.close()


class HttpServer:
    def __init__(self, servers: list):
        self.servers = servers

    async def serve_forever(self) -> None:
        await asyncio.gather(*(s.serve_forever() for s in self.servers))

    def close(self) -> None:
        for s in self.servers:
            s.close()


async def serve_http(svc, host: str, port: int, reuse_port: bool = False, backlog: int = 4096) -> HttpServer:
    loop = asyncio.get_running_loop()
    srv = await loop.create_server(lambda: HttpProtocol(svc), host, port, reuse_address=True,
                                   reuse_port=reuse_port or None, backlog=backlog, start_serving=True)
    return HttpServer([srv])
