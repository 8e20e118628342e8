"""Native asyncio HTTP/1.1 server of the OpenAI frontend (llm/http_server.py)
over real sockets: SSE streaming with chunked encoding, keep-alive +
pipelining, Expect: 100-continue, chunked request bodies, 404/405, client
disconnect stopping generation, SO_REUSEPORT."""
import asyncio
import json
import socket

import httpx

from dynamo_exp_amd.llm.backend import Backend
from dynamo_exp_amd.llm.engines import EchoEngineCore
from dynamo_exp_amd.llm.http_service import HttpService, RequestTemplate
from dynamo_exp_amd.llm.pipeline import LocalPipeline
from dynamo_exp_amd.llm.preprocessor import OpenAIPreprocessor
from dynamo_exp_amd.llm.tokenizer import SyntheticTokenizer


def run(coro, t=60):
    return asyncio.run(asyncio.wait_for(coro, t))


def _svc(**kw):
    tok = SyntheticTokenizer(1024, 0, [1])
    pre = OpenAIPreprocessor("echo", tok, eos_token_ids=[1])
    svc = HttpService("127.0.0.1", 0, request_template=RequestTemplate(model="echo", max_completion_tokens=64), **kw)
    svc.manager.add_chat_model("echo", LocalPipeline(pre, Backend(tok), EchoEngineCore()))
    svc.manager.add_completion_model("echo", LocalPipeline(pre, Backend(tok), EchoEngineCore()))
    return svc


def test_native_http_stream_unary_and_errors(monkeypatch):
    monkeypatch.setenv("DYN_TOKEN_ECHO_DELAY_MS", "0")
    svc = _svc()

    async def main():
        task = await svc.start_background()
        url = f"http://127.0.0.1:{svc.port}"
        try:
            async with httpx.AsyncClient(base_url=url, timeout=10) as c:
                r = await c.get("/v1/models")
                assert r.status_code == 200 and r.json()["data"][0]["id"] == "echo"
                assert (await c.get("/health")).json()["status"] == "healthy"
                r = await c.post("/v1/completions", json={"prompt": "hello world", "max_tokens": 100})
                assert r.status_code == 200 and r.json()["choices"][0]["text"] == "hello world"
                assert r.headers["x-request-id"]
                # SSE over chunked transfer-encoding, same connection (keep-alive)
                async with c.stream("POST", "/v1/chat/completions", headers={"x-request-id": "rid-1"},
                                    json={"stream": True, "messages": [{"role": "user", "content": "ping"}],
                                          "stream_options": {"include_usage": True}}) as s:
                    assert s.headers["content-type"].startswith("text/event-stream")
                    assert s.headers["x-request-id"] == "rid-1"
                    lines = [l async for l in s.aiter_lines() if l.startswith("data: ")]
                assert lines[-1] == "data: [DONE]"
                chunks = [json.loads(l[6:]) for l in lines[:-1]]
                assert chunks[0]["choices"][0]["delta"]["role"] == "assistant"
                assert "ping" in "".join(ch["choices"][0]["delta"].get("content") or "" for ch in chunks[:-1])
                assert chunks[-1]["usage"]["completion_tokens"] > 0
                r = await c.post("/v1/chat/completions", json={"model": "nope", "messages": []})
                assert r.status_code == 404
                r = await c.post("/v1/chat/completions", content=b"{not json")
                assert r.status_code == 400
                assert (await c.get("/v1/chat/completions")).status_code == 405
                assert (await c.get("/nothing")).status_code == 404
                m = (await c.get("/metrics")).text
                assert 'model="echo",request_type="stream",status="success"' in m
        finally:
            svc.stop()
            task.cancel()

    run(main())


def test_native_http_pipelining_continue_and_chunked_body(monkeypatch):
    monkeypatch.setenv("DYN_TOKEN_ECHO_DELAY_MS", "0")
    svc = _svc()

    async def main():
        task = await svc.start_background()
        port = svc.port
        try:
            body = json.dumps({"prompt": "abc", "max_tokens": 10}).encode()
            one = (b"POST /v1/completions HTTP/1.1\r\nhost: x\r\ncontent-type: application/json\r\n"
                   b"content-length: %d\r\n\r\n%b" % (len(body), body))
            # two pipelined requests on one connection: both answered, in order
            r, w = await asyncio.open_connection("127.0.0.1", port)
            w.write(one + one)
            got = b""
            while got.count(b'"text": "abc"') < 2:
                got += await asyncio.wait_for(r.read(65536), 10)
            assert got.count(b"HTTP/1.1 200 OK") == 2
            # Expect: 100-continue -> interim response before the body is sent
            w.write(b"POST /v1/completions HTTP/1.1\r\nhost: x\r\nexpect: 100-continue\r\n"
                    b"content-length: %d\r\n\r\n" % len(body))
            assert (await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 10)).startswith(b"HTTP/1.1 100 Continue")
            w.write(body)
            got = b""
            while b'"text": "abc"' not in got:
                got += await asyncio.wait_for(r.read(65536), 10)
            # chunked request body
            w.write(b"POST /v1/completions HTTP/1.1\r\nhost: x\r\ntransfer-encoding: chunked\r\n\r\n"
                    b"%x\r\n%b\r\n%x\r\n%b\r\n0\r\n\r\n" % (5, body[:5], len(body) - 5, body[5:]))
            got = b""
            while b'"text": "abc"' not in got:
                got += await asyncio.wait_for(r.read(65536), 10)
            # Connection: close is honoured
            w.write(b"GET /live HTTP/1.1\r\nhost: x\r\nconnection: close\r\n\r\n")
            got = b""
            while True:
                c = await asyncio.wait_for(r.read(65536), 10)
                if not c:
                    break
                got += c
            assert b"connection: close" in got and b'"live"' in got
            w.close()
        finally:
            svc.stop()
            task.cancel()

    run(main())


def test_native_http_client_disconnect_stops_generation(monkeypatch):
    monkeypatch.setenv("DYN_TOKEN_ECHO_DELAY_MS", "20")  # a slow stream the client walks away from
    svc = _svc()

    async def main():
        task = await svc.start_background()
        try:
            body = json.dumps({"stream": True, "max_tokens": 64,
                               "messages": [{"role": "user", "content": "a fairly long prompt " * 4}]}).encode()
            r, w = await asyncio.open_connection("127.0.0.1", svc.port)
            w.write(b"POST /v1/chat/completions HTTP/1.1\r\nhost: x\r\ncontent-length: %d\r\n\r\n%b"
                    % (len(body), body))
            got = b""
            while got.count(b"data: ") < 3:
                got += await asyncio.wait_for(r.read(65536), 10)
            w.close()
            g = svc.metrics.inflight.labels("echo")
            for _ in range(100):
                if g._value.get() == 0:
                    break
                await asyncio.sleep(0.05)
            assert g._value.get() == 0
            m = svc.metrics_text()
            assert 'status="cancelled"' in m
        finally:
            svc.stop()
            task.cancel()

    run(main())


def test_native_http_reuse_port_two_servers(monkeypatch):
    monkeypatch.setenv("DYN_TOKEN_ECHO_DELAY_MS", "0")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    a, b = _svc(reuse_port=True), _svc(reuse_port=True)
    a.port = b.port = port

    async def main():
        ta = await a.start_background()
        tb = await b.start_background()
        try:
            async with httpx.AsyncClient(base_url=f"http://127.0.0.1:{port}", timeout=10) as c:
                for _ in range(4):
                    assert (await c.get("/live")).status_code == 200
        finally:
            a.stop()
            b.stop()
            ta.cancel()
            tb.cancel()

    run(main())


def test_observe_many_matches_observe():
    """Batched histogram updates (the frontend's per-chunk ITL) export exactly what per-value observe() does."""
    import random
    import re

    from prometheus_client import CollectorRegistry, Histogram, generate_latest

    from dynamo_exp_amd.llm.http_service import observe_many

    b = [.001, .0025, .005, .01, .02, .04, .08, .16, .32, 1]
    r1, r2 = CollectorRegistry(), CollectorRegistry()
    h1 = Histogram("x", "x", ["m"], buckets=b, registry=r1).labels("a")
    h2 = Histogram("x", "x", ["m"], buckets=b, registry=r2).labels("a")
    rng = random.Random(0)
    vals = [rng.random() * 0.5 for _ in range(500)] + [0.01, 0.08, 1.0, 5.0]
    for v in vals:
        h1.observe(v)
    observe_many(h2, vals[:200])
    observe_many(h2, vals[200:])
    strip = lambda t: re.sub(r"x_created.*\n", "", t.decode())  # noqa: E731
    a, c = strip(generate_latest(r1)), strip(generate_latest(r2))
    assert [l for l in a.splitlines() if "_sum" not in l] == [l for l in c.splitlines() if "_sum" not in l]
    sa = float(re.search(r'x_sum\{m="a"\} (\S+)', a).group(1))
    sc = float(re.search(r'x_sum\{m="a"\} (\S+)', c).group(1))
    assert abs(sa - sc) < 1e-9 * max(1.0, sa)


def test_native_http_huge_chunk_header_refused_early(monkeypatch):
    """a chunk whose declared size exceeds MAX_BODY is
    refused with 413 as soon as its size line arrives, before its bytes are
    buffered."""
    monkeypatch.setenv("DYN_TOKEN_ECHO_DELAY_MS", "0")
    svc = _svc()

    async def main():
        task = await svc.start_background()
        try:
            r, w = await asyncio.open_connection("127.0.0.1", svc.port)
            w.write(b"POST /v1/completions HTTP/1.1\r\nhost: x\r\ntransfer-encoding: chunked\r\n\r\n"
                    b"%x\r\nabc" % (1 << 40))
            got = await asyncio.wait_for(r.read(65536), 10)
            assert got.startswith(b"HTTP/1.1 413")
            w.close()
        finally:
            svc.stop()
            task.cancel()

    run(main())


def test_native_http_stream_failure_closes_connection(monkeypatch):
    """a stream that raises after the chunked SSE head was
    written leaves an unterminated response; the server must close the
    connection (the client sees EOF) instead of keeping it alive."""
    from dynamo_exp_amd.llm import http_server

    monkeypatch.setenv("DYN_TOKEN_ECHO_DELAY_MS", "0")
    svc = _svc()

    class Boom:
        status, headers, body = 200, {}, None

        def __init__(self):
            async def gen():
                yield b"data: {}\n\n"
                raise RuntimeError("engine died mid-stream")
            self.stream = gen()

    async def handle(ep, body, headers):
        return Boom()

    async def main():
        task = await svc.start_background()
        monkeypatch.setattr(svc, "handle", handle)
        try:
            r, w = await asyncio.open_connection("127.0.0.1", svc.port)
            body = b'{"prompt": "x", "stream": true}'
            w.write(b"POST /v1/completions HTTP/1.1\r\nhost: x\r\ncontent-length: %d\r\n\r\n%b" % (len(body), body))
            got = b""
            while True:
                c = await asyncio.wait_for(r.read(65536), 10)
                if not c:
                    break  # EOF: the server closed the connection
                got += c
            assert got.startswith(b"HTTP/1.1 200") and b"0\r\n\r\n" not in got
        finally:
            svc.stop()
            task.cancel()

    assert http_server.MAX_BODY > 0
    run(main())
