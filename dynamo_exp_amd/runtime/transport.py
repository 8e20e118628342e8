"""Request plane: streaming RPC between components.

Reference design: a NATS request carries a
two-part message, then the worker opens a *new TCP connection back* to the
caller for every response stream.  Here each serving process runs one
`EndpointServer`; callers keep one persistent, multiplexed connection per
server (no per-request connect on the TTFT path).  Frames are the reference's
two-part frames (xxh3 checksummed, `_C_runtime` codec) with msgpack header and
body.

  caller -> server   {t: req,  id, ep}  body=request      |  {t: stop|kill, id}
                     {t: stats, id}                       (service stats scrape)
  server -> caller   {t: prologue, id, error?}            (error => stream fails)
                     {t: data, id} body=item  ...  {t: end, id}  |  {t: err, id, error}

Semantics kept from the reference: errors travel in the prologue, stop is a
graceful request to the producer (Context.stop_generating), kill drops the
stream, a failed send stops generation, and the server tracks in-flight
requests for graceful drain (push_endpoint.rs:55-106).
"""
from __future__ import annotations

import asyncio
import inspect
import itertools
import logging
import os
import socket
from typing import Any, AsyncIterator, Awaitable, Callable

import msgpack

from ..utils.tracing import stage
from .chan import Chan
from .context import Context
from .wire import TwoPartError, encode_two_part, iter_two_part

# bytes queued in a connection's transport before a sender waits for the socket
_HIGH_WATER = 1 << 20

log = logging.getLogger("dynamo_exp_amd.transport")


def _dumps(obj) -> bytes:
    if hasattr(obj, "model_dump"):
        obj = obj.model_dump()
    return msgpack.packb(obj, use_bin_type=True, default=_default)


def _default(o):
    if hasattr(o, "model_dump"):
        return o.model_dump()
    if hasattr(o, "tolist"):
        return o.tolist()
    if isinstance(o, (set, tuple)):
        return list(o)
    raise TypeError(f"cannot serialize {type(o)}")


def _loads(b: bytes):
    return msgpack.unpackb(b, raw=False, strict_map_key=False)


class _Cork:
    """Frames written during one event-loop iteration leave in ONE socket
    write (flushed by a call_soon callback): with hundreds of multiplexed
    streams each engine step turns into a burst of small frames on the same
    connection, and a send() syscall per frame was the top cost of the
    processor.  The flush runs after the callbacks already queued in this
    iteration, so the added latency is bounded by one loop iteration."""

    __slots__ = ("writer", "parts", "nbytes", "armed", "loop")

    def __init__(self, writer: asyncio.StreamWriter):
        self.writer = writer
        self.parts: list[bytes] = []
        self.nbytes = 0
        self.armed = False
        self.loop = asyncio.get_running_loop()

    def write(self, frame: bytes) -> None:
        self.parts.append(frame)
        self.nbytes += len(frame)
        if not self.armed:
            self.armed = True
            self.loop.call_soon(self.flush)

    def flush(self) -> None:
        self.armed = False
        if not self.parts:
            return
        data = self.parts[0] if len(self.parts) == 1 else b"".join(self.parts)
        self.parts = []
        self.nbytes = 0
        if not self.writer.is_closing():
            self.writer.write(data)

    def backlog(self) -> int:
        return self.nbytes + self.writer.transport.get_write_buffer_size()


# data-frame headers ({"t": "data", "id": sid}) repeat for every token of a
# stream: decode each distinct one once (read-only dicts)
_HCACHE: dict[bytes, dict] = {}


def _header(hb: bytes) -> dict:
    h = _HCACHE.get(hb)
    if h is None:
        h = _loads(hb)
        if h.get("t") == "data" and len(h) == 2:
            if len(_HCACHE) >= 1 << 16:
                _HCACHE.clear()
            _HCACHE[hb] = h
    return h


def local_ip() -> str:
    ip = os.environ.get("DX_HOST_IP")
    if ip:
        return ip
    return "127.0.0.1"


class EndpointError(Exception):
    pass


Handler = Callable[..., AsyncIterator[Any]]


class EndpointServer:
    """One per process: hosts every endpoint this process serves."""

    def __init__(self, host: str | None = None, port: int = 0):
        self.host = host or os.environ.get("DX_LISTEN_HOST", "0.0.0.0")
        self.port = port
        self.handlers: dict[str, tuple[Handler, bool]] = {}
        self.stats_handlers: dict[str, Callable[[], Any]] = {}
        self.inflight: dict[str, int] = {}
        self._server: asyncio.AbstractServer | None = None
        self._drain_waiters: dict[str, asyncio.Event] = {}
        self.accepting: dict[str, bool] = {}

    async def start(self) -> "EndpointServer":
        if self._server is None:
            self._server = await asyncio.start_server(self._conn, self.host, self.port, limit=1 << 26)
            self.port = self._server.sockets[0].getsockname()[1]
        return self

    @property
    def address(self) -> str:
        return f"{local_ip()}:{self.port}"

    def register(self, path: str, handler: Handler, stats_handler=None) -> None:
        params = list(inspect.signature(handler).parameters)
        wants_ctx = len(params) >= 2
        self.handlers[path] = (handler, wants_ctx)
        self.inflight.setdefault(path, 0)
        self.accepting[path] = True
        if stats_handler is not None:
            self.stats_handlers[path] = stats_handler

    def unregister(self, path: str) -> None:
        self.accepting[path] = False

    async def drain(self, path: str, timeout: float = 30.0) -> None:
        """Stop accepting `path` and wait for its in-flight requests."""
        self.accepting[path] = False
        end = asyncio.get_running_loop().time() + timeout
        while self.inflight.get(path, 0) > 0 and asyncio.get_running_loop().time() < end:
            await asyncio.sleep(0.02)
        self.handlers.pop(path, None)

    async def stop(self) -> None:
        if self._server is not None:
            self._server.close()
            await self._server.wait_closed()
            self._server = None

    async def _conn(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        sock = writer.get_extra_info("socket")
        if sock is not None:
            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        lock = asyncio.Lock()
        ctxs: dict[int, Context] = {}
        tasks: dict[int, asyncio.Task] = {}
        cork = _Cork(writer)

        def put(h: dict | bytes, body: bytes = b"") -> bool:
            """Cork one frame; True when the socket is backed up.  `h` may
            be a pre-encoded header (a stream's data frames)."""
            if writer.is_closing():
                raise ConnectionResetError("request plane connection closed")
            cork.write(encode_two_part(h if isinstance(h, bytes) else _dumps(h), body))
            return cork.backlog() > _HIGH_WATER

        async def send(h: dict | bytes | None, body: bytes = b"") -> None:
            # frames of every stream on this connection are corked per loop
            # iteration (no await); only a backed-up socket makes a sender
            # wait (one drainer at a time).  h=None: just wait for the drain
            if (h is None or put(h, body)) and cork.backlog() > _HIGH_WATER:
                async with lock:
                    cork.flush()
                    await writer.drain()

        send.put = put

        try:
            async for hb, body in iter_two_part(reader):
                h = _loads(hb)
                t, sid = h.get("t"), h.get("id")
                if t == "req":
                    ctx = Context(h.get("rid"), h.get("meta") or {})
                    ctxs[sid] = ctx
                    tasks[sid] = asyncio.create_task(self._serve(h.get("ep"), sid, body, ctx, send, ctxs, tasks))
                elif t in ("stop", "kill"):
                    c = ctxs.get(sid)
                    if c is not None:
                        c.kill() if t == "kill" else c.stop_generating()
                        if t == "kill" and sid in tasks:
                            tasks[sid].cancel()
                elif t == "stats":
                    out = {}
                    for p, fn in self.stats_handlers.items():
                        try:
                            r = fn()
                            if inspect.isawaitable(r):
                                r = await r
                            out[p] = r
                        except Exception as e:  # noqa: BLE001
                            out[p] = {"error": str(e)}
                    await send({"t": "stats", "id": sid, "stats": out,
                                "inflight": dict(self.inflight)})
                elif t == "ping":
                    await send({"t": "pong", "id": sid})
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        except (TwoPartError, msgpack.exceptions.ExtraData, ValueError) as e:
            # a corrupt frame (checksum / length / header) poisons the byte
            # stream: drop the connection cleanly, the client reconnects
            peer = writer.get_extra_info("peername")
            log.warning("request plane: closing connection from %s after a bad frame: %s", peer, e)
        finally:
            for c in ctxs.values():
                c.kill()
            for tk in tasks.values():
                tk.cancel()
            writer.close()

    async def _serve(self, path, sid, body, ctx, send, ctxs, tasks) -> None:
        entry = self.handlers.get(path)
        if entry is None or not self.accepting.get(path, False):
            await send({"t": "prologue", "id": sid, "error": f"endpoint {path} not served here"})
            ctxs.pop(sid, None)
            tasks.pop(sid, None)
            return
        handler, wants_ctx = entry
        stage(f"srv.recv:{path}", ctx.id)
        self.inflight[path] = self.inflight.get(path, 0) + 1
        try:
            try:
                req = _loads(body)
                gen = handler(req, ctx) if wants_ctx else handler(req)
                if inspect.isawaitable(gen) and not hasattr(gen, "__aiter__"):
                    gen = await gen
            except Exception as e:  # noqa: BLE001
                log.exception("handler setup failed")
                await send({"t": "prologue", "id": sid, "error": f"{type(e).__name__}: {e}"})
                return
            await send({"t": "prologue", "id": sid})

            async def emit(h, b=b""):
                try:
                    await send(h, b)
                except (ConnectionError, RuntimeError) as e:  # caller went away
                    raise _SendFailed() from e

            data_h = _dumps({"t": "data", "id": sid})
            try:
                if hasattr(gen, "__aiter__"):
                    first = True
                    killed = ctx.is_killed
                    async for item in gen:
                        if killed():
                            break
                        if first:
                            first = False
                            stage(f"srv.first:{path}", ctx.id)
                        # the frame is corked synchronously; await only when the socket backs up
                        try:
                            backed_up = send.put(data_h, _dumps(item))
                        except (ConnectionError, RuntimeError) as e:
                            raise _SendFailed() from e
                        if backed_up:
                            await emit(None)
                else:  # unary handler returned a value
                    await emit(data_h, _dumps(gen))
                await emit({"t": "end", "id": sid})
            except _SendFailed:
                ctx.stop_generating()  # a failed send stops generation (reference push_handler.rs:104)
            except asyncio.CancelledError:
                ctx.kill()
            except Exception as e:  # noqa: BLE001
                log.exception("handler failed")
                try:
                    await send({"t": "err", "id": sid, "error": f"{type(e).__name__}: {e}"})
                except Exception:
                    pass
            finally:
                if hasattr(gen, "aclose"):
                    try:
                        await gen.aclose()
                    except Exception:
                        pass
        finally:
            self.inflight[path] -= 1
            ctxs.pop(sid, None)
            tasks.pop(sid, None)


class _SendFailed(Exception):
    pass


class _Conn:
    """Caller-side multiplexed connection to one EndpointServer."""

    def __init__(self, address: str):
        self.address = address
        self.reader = self.writer = None
        self.lock = asyncio.Lock()
        self.streams: dict[int, Chan] = {}
        self.ids = itertools.count(1)
        self.task = None
        self.alive = False

    async def open(self) -> "_Conn":
        host, port = self.address.rsplit(":", 1)
        self.reader, self.writer = await asyncio.open_connection(host, int(port), limit=1 << 26)
        sock = self.writer.get_extra_info("socket")
        if sock is not None:
            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        self.alive = True
        self.cork = _Cork(self.writer)
        self.task = asyncio.create_task(self._read())
        return self

    async def _read(self) -> None:
        try:
            async for hb, body in iter_two_part(self.reader):
                h = _header(hb)
                q = self.streams.get(h.get("id"))
                if q is not None:
                    q.put_nowait((h, body))
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.CancelledError):
            pass
        except (TwoPartError, msgpack.exceptions.ExtraData, ValueError) as e:
            log.warning("request plane: dropping connection after a bad frame: %s", e)
        finally:
            self.alive = False
            for q in self.streams.values():
                q.put_nowait(({"t": "err", "error": "connection lost"}, b""))
            if self.writer is not None:
                self.writer.close()

    async def send(self, h: dict, body: bytes = b"") -> None:
        self.cork.write(encode_two_part(_dumps(h), body))
        if self.cork.backlog() > _HIGH_WATER:
            async with self.lock:
                self.cork.flush()
                await self.writer.drain()

    async def close(self):
        if self.writer:
            self.writer.close()
        if self.task:
            self.task.cancel()


class ConnectionPool:
    def __init__(self):
        self.conns: dict[str, _Conn] = {}
        self._locks: dict[str, asyncio.Lock] = {}

    async def get(self, address: str) -> _Conn:
        c = self.conns.get(address)
        if c is not None and c.alive:
            return c
        lk = self._locks.setdefault(address, asyncio.Lock())
        async with lk:
            c = self.conns.get(address)
            if c is None or not c.alive:
                c = await _Conn(address).open()
                self.conns[address] = c
        return c

    async def close(self):
        for c in self.conns.values():
            await c.close()
        self.conns.clear()


class ResponseStream:
    """Async iterator over one remote response stream; supports stop/kill."""

    def __init__(self, conn: _Conn, sid: int, q: Chan, context: Context | None, path: str = ""):
        self.conn, self.sid, self.q, self.path = conn, sid, q, path
        self.context = context or Context()
        self._done = False
        self._first = True
        self.context.on_stop(self._on_stop)

    def _on_stop(self):
        if not self._done and self.conn.alive:
            t = "kill" if self.context.is_killed() else "stop"
            asyncio.ensure_future(self.conn.send({"t": t, "id": self.sid}))

    def __aiter__(self):
        return self

    async def __anext__(self):
        if self._done:
            raise StopAsyncIteration
        h, body = await self.q.get()
        t = h.get("t")
        if t == "data":
            if self._first:
                self._first = False
                stage(f"cli.first:{self.path}", self.context.id)
            return _loads(body)
        self._finish()
        if t == "end":
            raise StopAsyncIteration
        raise EndpointError(h.get("error", "stream failed"))

    def _finish(self):
        self._done = True
        self.conn.streams.pop(self.sid, None)

    async def aclose(self):
        if not self._done:
            self.context.kill()
            self._finish()


async def call_endpoint(pool: ConnectionPool, address: str, path: str, request: Any,
                        context: Context | None = None) -> ResponseStream:
    conn = await pool.get(address)
    sid = next(conn.ids)
    q = Chan()
    conn.streams[sid] = q
    ctx = context or Context()
    stage(f"cli.send:{path}", ctx.id)
    await conn.send({"t": "req", "id": sid, "ep": path, "rid": ctx.id, "meta": ctx.metadata}, _dumps(request))
    h, _ = await q.get()
    if h.get("t") != "prologue" or h.get("error"):
        conn.streams.pop(sid, None)
        raise EndpointError(h.get("error") or f"bad prologue {h}")
    return ResponseStream(conn, sid, q, ctx, path)


async def scrape_stats(pool: ConnectionPool, address: str, timeout: float = 0.3) -> dict | None:
    try:
        conn = await asyncio.wait_for(pool.get(address), timeout)
        sid = next(conn.ids)
        q = Chan()
        conn.streams[sid] = q
        await conn.send({"t": "stats", "id": sid})
        h, _ = await asyncio.wait_for(q.get(), timeout)
        conn.streams.pop(sid, None)
        return h.get("stats")
    except (asyncio.TimeoutError, OSError, EndpointError):
        return None
